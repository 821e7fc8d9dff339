#!/bin/bash
# Llama-3-70B fp8 decode at B = 1, 32k context: kernel trace (TP=1).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3r
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p70 -o run -- \
  python3 tools/bench_decode.py --model llama3-70b --dtype fp8 --ctx 32000 --batches 1 --new 48 > gpurun_out/r3r/p70.log 2>&1 || exit 1
python3 tools/trace_gaps.py /tmp/p70 > gpurun_out/r3r/p70_gaps.txt 2>&1
head -24 gpurun_out/r3r/p70_gaps.txt
grep "^{" gpurun_out/r3r/p70.log
