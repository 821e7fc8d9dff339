#!/bin/bash
# Round 4: decode attention plan in context class 1 (<= 12k) at B = 5 and 16, in situ (level-1 reduce shapes).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4n
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 5 --ctx 5800 --new 512 --rounds 2 \
  --variants plan,attnfused3,attnfused4,attnfused6,attnfused8 > gpurun_out/r4n/b5.jsonl 2> gpurun_out/r4n/b5.err \
  || { tail -20 gpurun_out/r4n/b5.err; exit 1; }
cat gpurun_out/r4n/b5.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 16 --ctx 5800 --new 512 --rounds 2 \
  --variants plan,attnfused2,attnfused3,attnfused4,attnsep3,attnsep4 > gpurun_out/r4n/b16.jsonl 2> gpurun_out/r4n/b16.err \
  || { tail -20 gpurun_out/r4n/b16.err; exit 1; }
cat gpurun_out/r4n/b16.jsonl
