#!/bin/bash
# Round 4: the class-1 attention plan keyed by graph bucket (6 fused splits), in situ, then the headline bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4q
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 10 --ctx 5800 --new 512 --rounds 2 \
  --variants plan,attnfused3,attnfused4,attnfused2 > gpurun_out/r4q/b10.jsonl 2> gpurun_out/r4q/b10.err \
  || { tail -20 gpurun_out/r4q/b10.err; exit 1; }
cat gpurun_out/r4q/b10.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 16 --ctx 5800 --new 512 --rounds 2 \
  --variants plan,attnfused2,attnfused4 > gpurun_out/r4q/b16.jsonl 2> gpurun_out/r4q/b16.err \
  || { tail -20 gpurun_out/r4q/b16.err; exit 1; }
cat gpurun_out/r4q/b16.jsonl
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/r4q/bench.json 2> gpurun_out/r4q/bench.err \
  || { tail -5 gpurun_out/r4q/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4q/bench.json')); print('bench', d['ms_per_step'], d['value'], d['phases_s'], d['reduce_plan'], d['timed_work'])"
