#!/bin/bash
# Round 4: the deferred RMSNorm row limit at the headline's real decode shapes (batch 39 in bucket 40, batch 10 in
# bucket 16), in situ.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4t
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 39 --ctx 4000 --new 256 --rounds 2 \
  --variants plan,defer40,defer64 > gpurun_out/r4t/b39.jsonl 2> gpurun_out/r4t/b39.err || { tail -20 gpurun_out/r4t/b39.err; exit 1; }
cat gpurun_out/r4t/b39.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 10 --ctx 5800 --new 384 --rounds 2 \
  --variants plan,defer0,defer8 > gpurun_out/r4t/b10.jsonl 2> gpurun_out/r4t/b10.err || { tail -20 gpurun_out/r4t/b10.err; exit 1; }
cat gpurun_out/r4t/b10.jsonl
