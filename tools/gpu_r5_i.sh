#!/bin/bash
# round 5: decode attention with up to 256 splits and the 8-wave register-streaming kernels (kernel tests),
# then in situ: the TP-shard attention plans at long contexts (70B fp8 TP=8 shard B=1 at 32k; 8B TP=8 shard
# B=1 at 13.5k) and the 4- vs 8-wave register-streaming workgroups (TP=8 shards and the TP=1 headline shapes)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode or skinny or fp8 or resid" > gpurun_out/r5_attn_tests.txt 2>&1 || exit $?
OUT=gpurun_out/r5_attn_plans_256.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,attnsep64,attnsep128,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 4000 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 10 --ctx 4000 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 13500 --variants plan,attnsep64,attnsep32 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 10 --ctx 6000 --variants plan,waves:4 >> $OUT 2>/dev/null || exit $?
cat $OUT
