#!/bin/bash
# fp8 gate_up + SwiGLU on 32x32 tiles: GEMM + parity + engine GPU tests, then BASELINE config 5.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/fp8m32
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_forward_parity_gpu.py tests/test_engine_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8m32/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fp8m32/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/bench_aggregator.py > gpurun_out/fp8m32/agg70.json 2> gpurun_out/fp8m32/agg70.err || { tail -5 gpurun_out/fp8m32/agg70.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/fp8m32/agg70.json')); print('config5', d['value'], d['prefill_s'], d['decode_ms_per_token'])"
