#!/bin/bash
# Round 4: decode attention plan at the level-1 reduce shape (B=10, ~6k context, context class <= 12k), in situ.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4m
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 10 --ctx 5800 --new 512 --rounds 2 \
  --variants plan,attnfused3,attnfused6,attnfused8,attnsep6,attnsep9,attnsep12 > gpurun_out/r4m/b10.jsonl 2> gpurun_out/r4m/b10.err \
  || { tail -20 gpurun_out/r4m/b10.err; exit 1; }
cat gpurun_out/r4m/b10.jsonl
