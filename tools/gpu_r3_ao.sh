#!/bin/bash
# In situ, TP=1 B=1 at 10k context (the final reduce): fused vs separate split merge.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ao
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 1 --ctx 10000 --rounds 2 \
  --variants plan,attnfused16,attnfused24,attnfused32,attnsep48,attnsep64 > gpurun_out/r3ao/b1.jsonl 2> gpurun_out/r3ao/b1.err || { tail -5 gpurun_out/r3ao/b1.err; exit 1; }
cat gpurun_out/r3ao/b1.jsonl
