#!/bin/bash
# Restored-container tree: full GPU suite + smoke() on the freshly rebuilt .so files.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/restored
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/restored/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/restored/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/restored/smoke.log 2>&1 || exit $?
echo smoke ok
