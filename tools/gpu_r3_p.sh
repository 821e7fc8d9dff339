#!/bin/bash
# TP=8 shard decode step across batch sizes 12..39 and a kernel trace at B=20.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3p
timeout -k 10 300 python tools/bench_decode.py --tp-shard 8 --batches 12,16,17,20,24,28,32,39 --new 128 2>/dev/null \
  > gpurun_out/r3p/steps.jsonl || exit 1
cat gpurun_out/r3p/steps.jsonl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8_20 -o run -- \
  python3 tools/bench_decode.py --batches 20 --new 128 --tp-shard 8 > gpurun_out/r3p/p8_b20.log 2>&1 || exit 1
python3 tools/trace_gaps.py /tmp/p8_20 > gpurun_out/r3p/p8_b20_gaps.txt 2>&1
head -16 gpurun_out/r3p/p8_b20_gaps.txt
