#!/bin/bash
# Multi-process rehearsal of the round-3 tree on one GPU: bench.py self-launching 2 ranks (gloo; ranks share
# cuda:0) under the planner (auto) and a fixed per-stage layout with a TP=2 stage, 1 h transcript, 64 tokens.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ad
export MRSUM_DP_KV_FRACTION=0.15 MRSUM_REDUCE_KV_FRACTION=0.15 ENGINE_KV_FRACTION=0.15 MRSUM_DIST_BACKEND=gloo
timeout -k 10 500 python bench.py --gpus 2 --hours 1 --steps 1 --warmup 1 --max-new-tokens 64 --parallel auto \
  > gpurun_out/r3ad/auto.json 2> gpurun_out/r3ad/auto.err || { tail -5 gpurun_out/r3ad/auto.err; exit 1; }
tail -n 1 gpurun_out/r3ad/auto.json
timeout -k 10 500 python bench.py --gpus 2 --hours 1 --steps 1 --warmup 1 --max-new-tokens 64 --parallel map:tp2,reduce:dp \
  > gpurun_out/r3ad/fixed.json 2> gpurun_out/r3ad/fixed.err || { tail -5 gpurun_out/r3ad/fixed.err; exit 1; }
tail -n 1 gpurun_out/r3ad/fixed.json
