#!/bin/bash
# In-situ plan experiments for the TP=8 shard at B=39 / 20 (the map phase on 8 GPUs at TP=8 / TP=4 x DP=2).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ac
timeout -k 10 500 python tools/exp_plans_insitu.py --tp-shard 8 --batch 39 --rounds 2 \
  --variants plan,attnsep12,attnsep18,attnfused6,attnfused12,down:stream:4:7,down:stream:8:14,o:stream:4:2,o:stream:8:4 \
  > gpurun_out/r3ac/b39.jsonl 2> gpurun_out/r3ac/b39.err || { tail -5 gpurun_out/r3ac/b39.err; exit 1; }
cat gpurun_out/r3ac/b39.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --tp-shard 8 --batch 20 --rounds 2 \
  --variants plan,attnsep12,attnsep24,attnfused12 > gpurun_out/r3ac/b20.jsonl 2> gpurun_out/r3ac/b20.err || { tail -5 gpurun_out/r3ac/b20.err; exit 1; }
cat gpurun_out/r3ac/b20.jsonl
