#!/bin/bash
# round 5: engine GPU tests incl. the pinned-window replay test
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r5_jj_engine_tests.txt 2>&1
rc=$?; echo "rc=$rc"; tail -n 4 gpurun_out/r5_jj_engine_tests.txt; exit $rc
