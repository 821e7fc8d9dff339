#!/bin/bash
# Staggered prefill attention (two barriers per tile, waves 4-7 half a tile behind) vs one barrier per tile.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3u
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py -k "prefill or long" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3u/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3u/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  MRSUM_ATTN_PREFILL_STAGGER=0 timeout -k 10 200 python tools/bench_attn_prefill.py --tag onebar >> gpurun_out/r3u/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag stagger >> gpurun_out/r3u/ab.jsonl || exit 1
  MRSUM_ATTN_PREFILL_STAGGER=0 timeout -k 10 200 python tools/bench_attn_prefill.py --tag onebar --hq 64 --hkv 8 --cases 1x32768 >> gpurun_out/r3u/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag stagger --hq 64 --hkv 8 --cases 1x32768 >> gpurun_out/r3u/ab.jsonl || exit 1
done
cat gpurun_out/r3u/ab.jsonl
