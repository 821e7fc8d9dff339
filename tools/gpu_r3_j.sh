#!/bin/bash
# Llama-3-70B fp8 decode at B = 1, in situ: the deferred-norm producers (o, down) and the 32k attention plan.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3j
OUT=gpurun_out/r3j/plans70.jsonl
: > $OUT
timeout -k 10 700 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --ctx 8000 --new 128 --variants \
plan,fp8resid:8192:8192:4:4,fp8resid:8192:8192:8:8,fp8resid:8192:8192:4:2,fp8resid:8192:28672:4:4,fp8resid:8192:28672:8:7,fp8resid:8192:28672:8:8,fp8resid:8192:28672:8:14 \
  2>/dev/null >> $OUT || exit 1
cat $OUT
timeout -k 10 600 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --ctx 32000 --new 128 --rounds 1 \
  --variants plan,attnfused32,attnsep64,attnsep48 2>/dev/null >> $OUT || exit 1
cat $OUT | tail -4
