#!/bin/bash
# 70B fp8 decode at 32k B=1 in situ: o / down deferred-norm producer (stream, x resident, split-K residual) configs.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3am
timeout -k 10 1000 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --ctx 32000 --batch 1 --new 64 --rounds 2 \
  --variants plan,fp8resid:8192:28672:8:2,fp8resid:8192:28672:4:2,fp8resid:8192:28672:8:8,fp8resid:8192:8192:8:2,fp8resid:8192:8192:4:4,fp8resid:8192:8192:4:2 \
  > gpurun_out/r3am/p70.jsonl 2> gpurun_out/r3am/p70.err || { tail -5 gpurun_out/r3am/p70.err; exit 1; }
cat gpurun_out/r3am/p70.jsonl
