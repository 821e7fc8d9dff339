#!/bin/bash
# Round 4: decode GEMM plans in situ at the headline's real decode shapes: level-1 (batch 10 in bucket 16, ~6k
# context) and map (batch 39 in bucket 40, ~4k).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4r
timeout -k 10 500 python tools/exp_plans_insitu.py --batch 10 --ctx 5800 --new 384 --rounds 2 \
  --variants plan,qkv:stream:4:4,qkv:stream:8:4,qkv:stream:6:2,qkv:stream:6:8,down:stream:4:7,down:stream:8:4,down:stream:4:8,env:MRSUM_RESID_SKINNY_O=0 \
  > gpurun_out/r4r/b10.jsonl 2> gpurun_out/r4r/b10.err || { tail -20 gpurun_out/r4r/b10.err; exit 1; }
cat gpurun_out/r4r/b10.jsonl
timeout -k 10 500 python tools/exp_plans_insitu.py --batch 39 --ctx 4000 --new 256 --rounds 2 \
  --variants plan,qkv:stream:4:4,qkv:stream:8:4,o:stream:8:4,o:stream:4:2,down:stream:8:4,down:stream:4:7 \
  > gpurun_out/r4r/b39.jsonl 2> gpurun_out/r4r/b39.err || { tail -20 gpurun_out/r4r/b39.err; exit 1; }
cat gpurun_out/r4r/b39.jsonl
