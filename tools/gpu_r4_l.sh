#!/bin/bash
# Round 4: fp8-KV decode attention with FEWER splits at large batches (MRSUM_KV8_SPLIT_MULT < 1), in situ.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4l
for rep in 1 2; do
  for m in 1 0.5 0.75; do
    MRSUM_KV8_SPLIT_MULT=$m timeout -k 10 200 python tools/bench_decode.py --kv-dtype fp8 --batches 39,20 --ctx 4400 --new 256 \
      > gpurun_out/r4l/m$m.$rep.jsonl 2> gpurun_out/r4l/m$m.$rep.err || { tail -20 gpurun_out/r4l/m$m.$rep.err; exit 1; }
    sed "s/^/mult=$m rep=$rep /" gpurun_out/r4l/m$m.$rep.jsonl
  done
done
