#!/bin/bash
# GQA-packed prefill attention: kernel tests, then old (HEAD~ tree in .ab_old) vs new throughput at the
# 8B (32:8) and 70B (64:8) head layouts, then the full GPU suite, smoke and a short headline bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3t
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py -k "prefill or long" -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3t/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3t/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag old) >> gpurun_out/r3t/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag new >> gpurun_out/r3t/ab.jsonl || exit 1
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag old --hq 64 --hkv 8 --cases 1x32768,4x8192) >> gpurun_out/r3t/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag new --hq 64 --hkv 8 --cases 1x32768,4x8192 >> gpurun_out/r3t/ab.jsonl || exit 1
done
MRSUM_ATTN_PREFILL_PRIO=0 timeout -k 10 200 python tools/bench_attn_prefill.py --tag new_noprio >> gpurun_out/r3t/ab.jsonl || exit 1
cat gpurun_out/r3t/ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3t/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r3t/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3t/smoke.log 2>&1 || exit $?
echo smoke ok
