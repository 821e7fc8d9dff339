#!/bin/bash
# One-call GPU verification: pytest -m gpu, smoke(), then the headline bench (STEPS/WARMUP).
# Every GPU step has its own time limit; the first failure ends the call.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/v/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/v/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 600 python bench.py --steps "${STEPS:-2}" --warmup "${WARMUP:-1}" \
  > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err || exit $?
cat gpurun_out/v/bench.json
