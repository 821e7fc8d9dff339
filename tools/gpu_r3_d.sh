#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_forward_parity_gpu.py -x -v -s --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "attn_decode or parity" > gpurun_out/r3d/tests.log 2>&1
rc=$?; grep -E "parity:|passed|failed" gpurun_out/r3d/tests.log | tail -6; [ $rc -eq 0 ] || exit $rc
TAG=sc1 bash tools/gpu_ab_so.sh
