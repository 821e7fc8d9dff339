#!/bin/bash
# round 5, final tree: the full GPU suite, smoke(), then a rocprofv3 kernel trace of one 10 h bench step
# (per-kernel summary of the headline on the round-5 kernels)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5_gpu_tests_final2.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" | tee -a gpurun_out/r5_gpu_tests_final2.txt; tail -n 2 gpurun_out/r5_gpu_tests_final2.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke_final2.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/r5_smoke_final2.txt
[ $rc -eq 0 ] || exit $rc
NAME=r5_e2e_prof TO=420 bash tools/gpu_prof.sh
