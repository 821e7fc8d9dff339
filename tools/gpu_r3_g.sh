#!/bin/bash
# Confirm the TP-shard plan changes in situ (new plan vs the previous choices), TP = 8 / 4 / 2 shards.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3g
OUT=gpurun_out/r3g/plans.jsonl
: > $OUT
run() { timeout -k 10 300 python tools/exp_plans_insitu.py "$@" 2>/dev/null >> $OUT || exit 1; }
run --tp-shard 8 --batch 1 --variants plan,attnsep32,attnsep48,attnfused16,o:stream:4:4,down:stream:8:7
run --tp-shard 8 --batch 10 --variants plan,attnfused16,o:stream:4:4,down:stream:8:7
run --tp-shard 4 --batch 1 --variants plan,attnfused16,attnsep32,o:stream:4:4
run --tp-shard 4 --batch 10 --variants plan,attnfused16,o:stream:4:4
run --tp-shard 2 --batch 1 --variants plan,attnfused16,o:stream:4:4
for tp in 8 4 2; do timeout -k 10 300 python tools/bench_decode.py --batches 1,10,39 --ctx 4000 --new 256 --tp-shard $tp 2>/dev/null >> $OUT || exit 1; done
cat $OUT
