#!/bin/bash
# round 5: config 5's prefill (Llama-3-70B fp8, 32k-token prompt) at chunked-prefill slice sizes 4096 (shipped) /
# 8192 / 16384, alternating on one box (MRSUM_PREFILL_CHUNK, read at engine start; 16 new tokens: prefill only)
set -uo pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_p_prefill_chunk_ab.jsonl
: > $OUT
for r in 1 2; do
  for c in 4096 8192 16384; do
    MRSUM_PREFILL_CHUNK=$c timeout -k 10 300 python -u tools/bench_aggregator.py --steps 1 --warmup 1 --max-new-tokens 16 \
      2>/dev/null | grep "^{" | sed "s|^{|{\"prefill_chunk\": $c, |" >> $OUT || exit 1
  done
done
cat $OUT
