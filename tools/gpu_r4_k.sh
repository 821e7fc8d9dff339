#!/bin/bash
# Round 4: PMC passes, gemm.hip vs gemm4w.hip vs hipBLASLt (own runs, kernel-trace only besides --pmc).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
timeout -s KILL 120 python3 tools/pmc_gemm_vs_blas.py > gpurun_out/r4k/plain.log 2>&1 || exit $?
i=0
for CTRS in "SQ_VALU_MFMA_BUSY_CYCLES:SQ_WAVE_CYCLES:SQ_BUSY_CYCLES:GRBM_GUI_ACTIVE" \
            "SQ_WAVE_CYCLES:SQ_WAIT_INST_LDS:SQ_WAIT_INST_ANY:SQ_WAIT_ANY:SQ_ACTIVE_INST_ANY:SQ_ACTIVE_INST_VALU:SQ_ACTIVE_INST_LDS:SQ_ACTIVE_INST_MISC" \
            "SQ_WAVE_CYCLES:SQ_LDS_BANK_CONFLICT:SQ_LDS_IDX_ACTIVE:SQ_INSTS_VALU:SQ_INSTS_LDS:SQ_INSTS_SALU:SQ_INSTS_SMEM" \
            "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/pk$i -o run -- \
    python3 tools/pmc_gemm_vs_blas.py > gpurun_out/r4k/pass$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/r4k/pass$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pk$i > gpurun_out/r4k/pass$i.txt 2>&1
  echo "== pass $i: $CTRS"; cut -c1-260 gpurun_out/r4k/pass$i.txt
done
