#!/bin/bash
# PMC passes over the prefill GEMM (own runs, kernel-trace only besides --pmc): MFMA busy, where wave time
# goes (SQ_WAIT_* / SQ_ACTIVE_*), LDS bank conflicts, beyond-L2 read bytes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/pmcgemm
export TMPDIR=/tmp
timeout -s KILL 120 python3 tools/pmc_gemm.py > gpurun_out/pmcgemm/plain.log 2>&1 || exit $?
i=0
for CTRS in "SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_WAVE_CYCLES:SQ_WAIT_INST_LDS:SQ_WAIT_INST_ANY:SQ_WAIT_ANY:SQ_ACTIVE_INST_ANY:SQ_ACTIVE_INST_VALU:SQ_ACTIVE_INST_LDS" \
            "SQ_WAVE_CYCLES:SQ_ACTIVE_INST_MISC:SQ_ACTIVE_INST_SCA:SQ_ACTIVE_INST_FLAT:SQ_LDS_BANK_CONFLICT:SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/pg$i -o run -- \
    python3 tools/pmc_gemm.py > gpurun_out/pmcgemm/pass$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmcgemm/pass$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pg$i > gpurun_out/pmcgemm/pass$i.txt 2>&1
  echo "== pass $i: $CTRS"; cat gpurun_out/pmcgemm/pass$i.txt
done
