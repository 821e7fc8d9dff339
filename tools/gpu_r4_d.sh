#!/bin/bash
# fp8 KV: decode-attention split multiplier sweep in situ (whole decode steps) at B = 10 / 39, 4.4k context.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4d
for m in 1 2 3; do
  MRSUM_KV8_SPLIT_MULT=$m timeout -k 10 300 python tools/bench_decode.py --batches 10,39,20 --ctx 4400 --new 128 --kv-dtype fp8 \
    > gpurun_out/r4d/m$m.jsonl 2> gpurun_out/r4d/m$m.err || { tail -5 gpurun_out/r4d/m$m.err; exit 1; }
  sed "s/^{/{\"kv8_split_mult\": $m, /" gpurun_out/r4d/m$m.jsonl >> gpurun_out/r4d/sweep.jsonl
done
cat gpurun_out/r4d/sweep.jsonl
