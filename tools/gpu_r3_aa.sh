#!/bin/bash
# PMC: fp8 vs bf16 stream GEMM at equal bytes / row length (own runs, kernel-trace only besides --pmc).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3aa
export TMPDIR=/tmp
timeout -s KILL 120 python3 tools/pmc_fp8_stream.py > gpurun_out/r3aa/plain.log 2>&1 || exit $?
i=0
for CTRS in "SQ_WAVE_CYCLES:SQ_WAIT_INST_LDS:SQ_WAIT_INST_ANY:SQ_WAIT_ANY:SQ_ACTIVE_INST_ANY:SQ_ACTIVE_INST_VALU:SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "SQ_WAVE_CYCLES:SQ_INSTS_VALU:SQ_INSTS_LDS:SQ_INSTS_SALU:SQ_INSTS_SMEM:SQ_INST_LEVEL_VMEM:SQ_WAVES"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/pf$i -o run -- \
    python3 tools/pmc_fp8_stream.py > gpurun_out/r3aa/pass$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/r3aa/pass$i.log; continue; }
  python3 tools/pmc_summary.py /tmp/pf$i > gpurun_out/r3aa/pass$i.txt 2>&1
  cat gpurun_out/r3aa/pass$i.txt
  find /tmp/pf$i -name "*counter_collection.csv" -exec cp {} gpurun_out/r3aa/pass$i.csv \;
done
