#!/bin/bash
# In situ, TP=1: decode attention split variants at B=10 (level-1 reduce) and B=5 / B=20, 4k context.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3an
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 10 --rounds 2 \
  --variants plan,attnfused4,attnfused6,attnfused8,attnsep6,attnsep9 > gpurun_out/r3an/b10.jsonl 2> gpurun_out/r3an/b10.err || { tail -5 gpurun_out/r3an/b10.err; exit 1; }
cat gpurun_out/r3an/b10.jsonl
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 20 --rounds 2 \
  --variants plan,attnfused3,attnfused4,attnfused6,attnsep4 > gpurun_out/r3an/b20.jsonl 2> gpurun_out/r3an/b20.err || { tail -5 gpurun_out/r3an/b20.err; exit 1; }
cat gpurun_out/r3an/b20.jsonl
