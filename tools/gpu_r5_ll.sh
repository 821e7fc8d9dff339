#!/bin/bash
# round 5, end of session: the full GPU suite and smoke() on the final tree
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5_gpu_tests_end.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" | tee -a gpurun_out/r5_gpu_tests_end.txt; tail -n 2 gpurun_out/r5_gpu_tests_end.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke_end.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/r5_smoke_end.txt; exit $rc
