#!/bin/bash
# Fused norm + fp8 quantisation: kernel test, fp8 parity, 70B fp8 32k aggregator pass (config 5) with the
# fused quant on / off, then the 70B B=1 decode trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3s
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_forward_parity_gpu.py -x -v --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "rmsnorm_fp8 or fp8" > gpurun_out/r3s/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r3s/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3_r.sh
