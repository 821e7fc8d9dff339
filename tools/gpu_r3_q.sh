#!/bin/bash
# TP push at every decode batch + the gate_up plan fix: tests, then the planner's decode-step set.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3q
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py -x -v --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "tp_push or tp2 or skinny_resid" > gpurun_out/r3q/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r3q/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3_n.sh
