#!/bin/bash
# round 5: decode-attention split / merge plans in situ (whole decode steps) with the four-register-set
# kernel: TP=1 B=1 at 13.5k (final reduce), TP=8 shard B=1 / 10 at 4k
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_attn_plans_deep.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,attnsep16,attnsep24,attnfused16,attnsep48 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --variants plan,attnsep16,attnsep32,attnfused16,attnfused8 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 10 --variants plan,attnsep8,attnfused8,attnfused4 >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,attnsep64,attnsep48 >> $OUT 2>/dev/null || exit $?
cat $OUT
