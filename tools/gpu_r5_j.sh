#!/bin/bash
# round 5: 8-wave register-streaming workgroups + the o projection merging the attention splits (one row of
# a TP shard) + decode attention up to 256 splits: kernel tests, then whole-step A/Bs in situ (one engine per
# shape, variants interleaved): TP=8 shards of Llama-3-8B (B=1 / 10 at 4k, B=1 at 13.5k), the 70B fp8 TP=8
# shard at 32k, and the TP=1 headline shapes (B=1 at 13.5k, B=10 at 6k)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode or skinny or fp8 or resid or consumer_merge" > gpurun_out/r5_j_tests.txt 2>&1 || exit $?
OUT=gpurun_out/r5_j_insitu.jsonl
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 4000 --variants plan,cmerge:0,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,attnsep64,attnsep128,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 10 --ctx 4000 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 13500 --variants plan,attnsep64,cmerge:1000000 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 10 --ctx 6000 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
cat $OUT
