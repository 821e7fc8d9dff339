#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3c
timeout -k 10 600 python tools/diag_parity.py > gpurun_out/r3c/diag.log 2>&1; rc=$?
cat gpurun_out/r3c/diag.log | grep "^{"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r3c/diag.log; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "not parity" > gpurun_out/r3c/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3c/gpu_tests.log; exit $rc
