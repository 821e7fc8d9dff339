#!/bin/bash
# Round 4: decode attention plan at the final-reduce shape (B = 1, ~13.5k context, class <= 32k), in situ.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4o
timeout -k 10 500 python tools/exp_plans_insitu.py --batch 1 --ctx 13000 --new 1000 --rounds 2 \
  --variants plan,attnsep16,attnsep24,attnsep48,attnsep64,attnfused16 > gpurun_out/r4o/b1.jsonl 2> gpurun_out/r4o/b1.err \
  || { tail -20 gpurun_out/r4o/b1.err; exit 1; }
cat gpurun_out/r4o/b1.jsonl
