#!/bin/bash
# TP=8 shard B=1 kernel traces with the TP push on and off (same box).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3l
export TMPDIR=/tmp
for push in 1 0; do
  MRSUM_TP_PUSH=$push timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8_$push -o run -- \
    python3 tools/bench_decode.py --batches 1 --new 128 --tp-shard 8 > gpurun_out/r3l/p8_$push.log 2>&1 || exit 1
  python3 tools/trace_summary.py /tmp/p8_$push > gpurun_out/r3l/p8_${push}_summary.txt 2>&1
  python3 tools/trace_gaps.py /tmp/p8_$push > gpurun_out/r3l/p8_${push}_gaps.txt 2>&1
done
head -14 gpurun_out/r3l/p8_1_gaps.txt
head -14 gpurun_out/r3l/p8_0_gaps.txt
