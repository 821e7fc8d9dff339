#!/bin/bash
# Round 4: hipBLASLt's kernel names / times for the prefill projections next to gemm.hip (rocprofv3 stats).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i/prof -o blas -- python3 tools/blas_kernel_names.py \
  > gpurun_out/r4i/blas.log 2>&1 || { tail -20 gpurun_out/r4i/blas.log; exit 1; }
find gpurun_out/r4i/prof -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/r4i/prof -name "*kernel_stats.csv"); do cut -c1-400 "$f" | head -20; done
