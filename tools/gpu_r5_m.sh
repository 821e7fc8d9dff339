#!/bin/bash
# round 5: in-situ plan A/Bs at one decode row (whole steps, variants interleaved): the TP=8 shard of
# Llama-3-8B at 4k (fused vs separate attention merge, qkv on the register-streaming kernel, 8-wave LM head)
# and the TP=1 final reduce at 13.5k
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_m_insitu.jsonl
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 4000 --variants plan,attnfused16,attnfused32,qkv:skinny:1:4,qkv:skinny:1:8,w8max:2048 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,qkv:skinny:1:2,w8max:2048,attnfused16 >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 10 --ctx 6000 --variants plan,attnfused8,attnfused9,attnfused12,attnsep9,attnsep12 >> $OUT 2>/dev/null || exit $?
cat $OUT
