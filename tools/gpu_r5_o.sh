#!/bin/bash
# round 5: the headline bench at the driver's length (20 timed steps, 5 warmup) on the final kernels, then the
# TP=8 shard decode steps re-profiled per kernel after this round's changes (rocprofv3 kernel traces)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_20steps.json 2> gpurun_out/r5_bench_20steps.err || exit $?
run() {  # name, bench_decode args...
  local NAME=$1; shift
  timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/bench_decode.py "$@" > gpurun_out/$NAME.log 2>&1 || return $?
  mkdir -p gpurun_out/$NAME
  python3 tools/trace_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  python3 tools/trace_gaps.py /tmp/$NAME > gpurun_out/$NAME/gaps.txt 2>&1
  grep "^{" gpurun_out/$NAME.log
}
run r5_tp8_8b_b1_after --tp-shard 8 --batches 1 --ctx 4000 --new 128 || exit $?
run r5_tp8_70b_b1_32k_after --model llama3-70b --dtype fp8 --tp-shard 8 --batches 1 --ctx 32000 --new 128 || exit $?
echo done
