#!/bin/bash
# round 5: TP=8 shard decode steps decomposed per kernel (rocprofv3 kernel traces of tools/bench_decode.py
# --tp-shard 8: one rank's shard shapes on one GPU, the P2P all-reduce over a group of one):
#   Llama-3-8B bf16 B = 1 / 10 at 4k, Llama-3-70B fp8 B = 1 at 32k
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name, bench_decode args...
  local NAME=$1; shift
  timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/bench_decode.py "$@" > gpurun_out/$NAME.log 2>&1 || return $?
  mkdir -p gpurun_out/$NAME
  python3 tools/trace_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  python3 tools/trace_gaps.py /tmp/$NAME > gpurun_out/$NAME/gaps.txt 2>&1
  grep "^{" gpurun_out/$NAME.log
}
run r5_tp8_8b_b1 --tp-shard 8 --batches 1 --ctx 4000 --new 128 || exit $?
run r5_tp8_8b_b10 --tp-shard 8 --batches 10 --ctx 4000 --new 128 || exit $?
run r5_tp8_70b_b1_32k --model llama3-70b --dtype fp8 --tp-shard 8 --batches 1 --ctx 32000 --new 128 || exit $?
# the same steps without the profiler (per-step wall time in the graph)
timeout -k 10 300 python3 tools/bench_decode.py --tp-shard 8 --batches 1,10 --ctx 4000 --new 256 > gpurun_out/r5_tp8_steps.jsonl 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_decode.py --model llama3-70b --dtype fp8 --tp-shard 8 --batches 1 --ctx 32000 --new 256 >> gpurun_out/r5_tp8_steps.jsonl 2>&1 || exit $?
echo done
