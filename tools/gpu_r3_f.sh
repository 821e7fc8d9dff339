#!/bin/bash
# In-situ plan sweeps after the sc1 last-arriver change: TP=8 shard B=1/10 (attention splits / merge,
# gate_up kernel), TP=1 B=1/10/39 (attention merge).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3f
OUT=gpurun_out/r3f/plans.jsonl
: > $OUT
run() { timeout -k 10 300 python tools/exp_plans_insitu.py "$@" 2>/dev/null >> $OUT || exit 1; }
run --tp-shard 8 --batch 1 --variants plan,attnfused32,attnfused64,attnsep64,attnfused8,gate_up:stream_split:4:4,gate_up:stream_split:7:8,o:skinny:1:1,down:skinny:1:2
run --tp-shard 8 --batch 10 --variants plan,attnfused8,attnfused24,attnsep25,gate_up:stream_split:4:4,gate_up:stream_split:7:8
run --batch 1 --variants plan,attnfused16,attnfused32,attnfused64
run --batch 10 --variants plan,attnfused4,attnfused6,attnsep3
run --batch 39 --variants plan,attnfused3,attnfused2,attnsep2
cat $OUT
