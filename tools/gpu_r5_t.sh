#!/bin/bash
# round 5: where a B=1 decode-attention wave's time goes (vs B=39): SQ wait / active-instruction shares and the
# VMEM in-flight level, one rocprofv3 --pmc pass over tools/pmc_attn_decode.py (kernel trace + --pmc only)
set -uo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NAME=r5_t_pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM \
  --output-format csv -d /tmp/$NAME -o run -- python3 tools/pmc_attn_decode.py > gpurun_out/$NAME.log 2>&1 || exit $?
mkdir -p gpurun_out/$NAME
python3 tools/pmc_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
cat gpurun_out/$NAME/summary.txt
NAME=r5_t_pmc2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  --output-format csv -d /tmp/$NAME -o run -- python3 tools/pmc_attn_decode.py > gpurun_out/$NAME.log 2>&1 || exit $?
mkdir -p gpurun_out/$NAME
python3 tools/pmc_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
cat gpurun_out/$NAME/summary.txt
