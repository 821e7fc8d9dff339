#!/bin/bash
# Round 4: a decode bucket of 10 / 12 for the level-1 reduce's batch of 10 (in situ, ~6k context).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4s
timeout -k 10 500 python tools/exp_plans_insitu.py --batch 10 --ctx 5800 --new 384 --rounds 3 \
  --variants plan,buckets:1+2+4+8+10+16,buckets:1+2+4+8+12+16 \
  > gpurun_out/r4s/b10.jsonl 2> gpurun_out/r4s/b10.err || { tail -20 gpurun_out/r4s/b10.err; exit 1; }
cat gpurun_out/r4s/b10.jsonl
