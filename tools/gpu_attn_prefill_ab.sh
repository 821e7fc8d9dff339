set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/pa
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py tests/test_engine_gpu.py -k "prefill or long or engine or chunk" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pa/t.log 2>&1
rc=$?; tail -2 gpurun_out/pa/t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd .ab_old && timeout -k 10 300 python ../tools/bench_attn_prefill.py --tag old) || exit 1
  timeout -k 10 300 python tools/bench_attn_prefill.py --tag new || exit 1
done
