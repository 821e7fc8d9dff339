#!/bin/bash
# B=1 decode attention split plans in situ at the real long-context shapes: the headline's final reduce
# (Llama-3-8B, ~13.5k) and config 5 (Llama-3-70B fp8, 32k).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4ab
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --new 256 --rounds 2 \
  --variants plan,attnsep24,attnsep40,attnsep48,attnsep64,attnfused16 > gpurun_out/r4ab/b1_13k5.jsonl \
  2> gpurun_out/r4ab/b1_13k5.err || { tail -5 gpurun_out/r4ab/b1_13k5.err; exit 1; }
cat gpurun_out/r4ab/b1_13k5.jsonl
timeout -k 10 600 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --batch 1 --ctx 32000 --new 128 \
  --rounds 2 --variants plan,attnsep24,attnsep48,attnsep64 > gpurun_out/r4ab/b1_70b_32k.jsonl \
  2> gpurun_out/r4ab/b1_70b_32k.err || { tail -5 gpurun_out/r4ab/b1_70b_32k.err; exit 1; }
cat gpurun_out/r4ab/b1_70b_32k.jsonl
