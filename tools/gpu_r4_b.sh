#!/bin/bash
# Round 4: TP parity against fp32 (2 and 4 ranks sharing the GPU) + the custom all-reduce recovery test, verbose.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4b
timeout -k 10 900 python -u -m pytest tests/test_tp_parity_gpu.py tests/test_custom_ar_gpu.py -m gpu -x -v -s \
  --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r4b/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|parity:|passed|failed" gpurun_out/r4b/tests.log | tail -20
exit $rc
