#!/bin/bash
# Software-pipelined prefill attention (QK^T(t+1) || exp(t), 3-stage ring) vs the committed one-barrier loop (.ab_old).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3w
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py -k "prefill or long" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3w/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag base) >> gpurun_out/r3w/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag pipe >> gpurun_out/r3w/ab.jsonl || exit 1
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag base --hq 64 --hkv 8 --cases 1x32768) >> gpurun_out/r3w/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag pipe --hq 64 --hkv 8 --cases 1x32768 >> gpurun_out/r3w/ab.jsonl || exit 1
done
cat gpurun_out/r3w/ab.jsonl
