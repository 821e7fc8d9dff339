#!/bin/bash
# round 5: B=1 decode attention (8 kv heads, G=4) kernel time vs split count at the headline's final-reduce
# context (13.5k) and at 32k -- separate and fused merges, rotating over 8 caches (tools/bench_attn_decode.py)
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_attn_decode.py --batches 1 --ctx 13500 --splits 16,24,32,48,64,96,128 > gpurun_out/r5_s_attn_b1_splits.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attn_decode.py --batches 1 --ctx 32000 --splits 16,24,32,48,64,96,128 >> gpurun_out/r5_s_attn_b1_splits.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attn_decode.py --batches 10,39 --ctx 4400 --splits auto,2,3,4,6,9 >> gpurun_out/r5_s_attn_b1_splits.jsonl 2>&1 || exit $?
cat gpurun_out/r5_s_attn_b1_splits.jsonl
# PMC passes over the decode attention alone (own runs: kernel trace + --pmc only)
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r5_s_counters.txt 2>&1
i=0
for CTRS in "FETCH_SIZE" "SQ_WAVES:SQ_WAVE_CYCLES:SQ_WAIT_INST_ANY:SQ_BUSY_CYCLES:SQ_INSTS_VMEM_RD:SQ_INSTS_LDS" "TCP_TCC_READ_REQ_LATENCY_sum:TCP_TCC_READ_REQ_sum"; do
  i=$((i + 1))
  NAME=r5_s_pmc$i
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/pmc_attn_decode.py > gpurun_out/$NAME.log 2>&1 || { echo "pass $i rc=$?"; continue; }
  mkdir -p gpurun_out/$NAME
  python3 tools/pmc_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  cat gpurun_out/$NAME/summary.txt
done
