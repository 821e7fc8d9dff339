#!/bin/bash
# rocprofv3 PMC passes (own runs, kernel-trace only besides --pmc) over tools/pmc_kernels.py:
#   pass 1: FETCH_SIZE -> HBM read bytes -> achieved TB/s per kernel
#   pass 2: SQ_VALU_MFMA_BUSY_CYCLES -> MFMA utilisation
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 180 python3 tools/pmc_kernels.py > gpurun_out/pmc_plain.log 2>&1 || exit $?
i=0
for CTRS in ${PASSES:-"FETCH_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES"}; do
  i=$((i + 1))
  NAME=pmc_pass$i
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/pmc_kernels.py > gpurun_out/$NAME.log 2>&1 || exit $?
  mkdir -p gpurun_out/$NAME
  python3 tools/pmc_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  cat gpurun_out/$NAME/summary.txt
done
