#!/bin/bash
# Round 4 final tree, part A: full GPU suite + smoke(); hipBLASLt kernel names for the prefill projections.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4final/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4final/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final/smoke.log 2>&1 || { tail -20 gpurun_out/r4final/smoke.log; exit 1; }
echo smoke ok; tail -3 gpurun_out/r4final/smoke.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4final/blas -o blas -- python3 tools/blas_kernel_names.py \
  > gpurun_out/r4final/blas.log 2>&1 || { tail -20 gpurun_out/r4final/blas.log; exit 1; }
for f in $(find gpurun_out/r4final/blas -name "*kernel_stats.csv"); do cut -c1-300 "$f" | head -12; done
