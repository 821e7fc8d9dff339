#!/bin/bash
# 70B fp8 decode at 32k B=1 in situ: gate_up + SwiGLU on the stream kernel (x resident) vs the register-streaming plan.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3al
timeout -k 10 900 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --ctx 32000 --batch 1 --new 64 --rounds 2 \
  --variants plan,env:MRSUM_FP8_STREAM_SWIGLU=1 > gpurun_out/r3al/p70.jsonl 2> gpurun_out/r3al/p70.err || { tail -5 gpurun_out/r3al/p70.err; exit 1; }
cat gpurun_out/r3al/p70.jsonl
