#!/bin/bash
# In situ: the TP=1 deferred RMSNorm (residual update + sums of squares in the o / down split-K epilogue,
# consumers scale their rows) at B=39 vs the two add + RMSNorm launches per layer (plan).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ah
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 39 --rounds 3 --variants plan,defer64 \
  > gpurun_out/r3ah/b39.jsonl 2> gpurun_out/r3ah/b39.err || { tail -5 gpurun_out/r3ah/b39.err; exit 1; }
cat gpurun_out/r3ah/b39.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 20 --rounds 2 --variants plan,defer64 \
  > gpurun_out/r3ah/b20.jsonl 2> gpurun_out/r3ah/b20.err || { tail -5 gpurun_out/r3ah/b20.err; exit 1; }
cat gpurun_out/r3ah/b20.jsonl
