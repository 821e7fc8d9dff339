#!/bin/bash
# TP=1 small-batch decode: kernel traces at B=1/10 and in-situ producer variants (skinny residual update
# without split-K for o / down).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3o
export TMPDIR=/tmp
for B in 1 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p1_$B -o run -- \
    python3 tools/bench_decode.py --batches $B --new 128 > gpurun_out/r3o/p1_b$B.log 2>&1 || exit 1
  python3 tools/trace_gaps.py /tmp/p1_$B > gpurun_out/r3o/p1_b${B}_gaps.txt 2>&1
  head -12 gpurun_out/r3o/p1_b${B}_gaps.txt
done
for B in 1 10; do
  timeout -k 10 400 python tools/exp_plans_insitu.py --batch $B --new 192 --variants \
    plan,env:MRSUM_RESID_SKINNY_O=1,env:MRSUM_RESID_SKINNY_DOWN=1 2>/dev/null >> gpurun_out/r3o/insitu.jsonl || exit 1
done
cat gpurun_out/r3o/insitu.jsonl
