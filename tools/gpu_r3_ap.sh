#!/bin/bash
# Standalone decode attention (q given, no fused RoPE / slab sums) at the bench's contexts, to compare with
# the in-situ kernel times of the bench profile.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ap
timeout -k 10 300 python tools/bench_attn_decode.py --batches 1 --ctx 10000 --splits auto,16,64 > gpurun_out/r3ap/b1.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/bench_attn_decode.py --batches 10,39 --ctx 4400 --splits auto > gpurun_out/r3ap/b39.jsonl 2>&1 || exit 1
cat gpurun_out/r3ap/b1.jsonl gpurun_out/r3ap/b39.jsonl | grep "^{"
