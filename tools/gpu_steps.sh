#!/bin/bash
# The one GPU-call driver: run each argument as one step, in order, each under its own time limit, each
# logging to gpurun_out/<TAG>_<n>.log; stop at the first step that fails (no retries, nothing after a
# fault / abort / time limit).  Replaces the per-call one-off scripts of rounds 3-5.
#
#   gpurun --timeout 900 -- 'TAG=r6a STEP_T=300 bash tools/gpu_steps.sh \
#       "python tools/bench_decode.py --tp-shard 8 --batches 1" "python bench.py --steps 1 --warmup 1"'
#
# STEP_T: seconds per step (default 300).  The command of every step is echoed into its log's first line,
# so each record under profiles/ traces back to its command.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-step}
T=${STEP_T:-300}
n=0
for cmd in "$@"; do
  n=$((n + 1))
  log="gpurun_out/${TAG}_${n}.log"
  echo "# $cmd" > "$log"
  echo "[$(date +%T)] step $n: $cmd"
  timeout -k 10 "$T" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "[$(date +%T)] step $n rc=$rc"
  tail -n 4 "$log"
  if [ $rc -ne 0 ]; then
    echo "stopping after step $n (rc=$rc)"
    exit $rc
  fi
done
