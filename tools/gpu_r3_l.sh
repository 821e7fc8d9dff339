#!/bin/bash
# TP=8 shard kernel traces (TP push on) at B = 1 and 10.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3l
export TMPDIR=/tmp
for B in 1 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8_$B -o run -- \
    python3 tools/bench_decode.py --batches $B --new 128 --tp-shard 8 > gpurun_out/r3l/p8_b$B.log 2>&1 || exit 1
  python3 tools/trace_gaps.py /tmp/p8_$B > gpurun_out/r3l/p8_b${B}_gaps.txt 2>&1
  head -14 gpurun_out/r3l/p8_b${B}_gaps.txt
done
