#!/bin/bash
# round 5: chunked-prefill slice size for Llama-3-8B bf16 (the headline's final reduce prompt ~13.5k tokens and
# a 32k prompt): 4096 (shipped) / 8192 / 16384, alternating on one box (prefill only: 16 new tokens)
set -uo pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_r_prefill_chunk_8b_ab.jsonl
: > $OUT
for r in 1 2; do
  for ctx in 13500 32000; do
    for c in 4096 8192 16384; do
      MRSUM_PREFILL_CHUNK=$c timeout -k 10 300 python -u tools/bench_aggregator.py --model llama3-8b --dtype bf16 \
        --context $ctx --steps 2 --warmup 1 --max-new-tokens 16 2>/dev/null | grep "^{" | sed "s|^{|{\"prefill_chunk\": $c, |" >> $OUT || exit 1
    done
  done
done
cat $OUT
