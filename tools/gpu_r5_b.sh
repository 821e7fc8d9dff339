#!/bin/bash
# round 5 experiments: K/V prefetch A/B (B=1 at 13.5k: the headline's final reduce; B=5 at 4.4k: a DP=8
# map rank), fp8v vs bf16 vs fp8 KV decode steps at the map's B=39 / level-1 B=10 shapes
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for kv in bf16 fp8v fp8; do
  timeout -k 10 300 python -u tools/bench_decode.py --batches 39,10 --ctx 4400 --new 200 --kv-dtype $kv >> gpurun_out/r5_decode_kvfmt.jsonl 2>>gpurun_out/r5_decode_kvfmt.err || exit $?
done
echo done
