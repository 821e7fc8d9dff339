#!/bin/bash
# Config 5 (Llama-3-70B fp8 aggregator, ~32k context, TP=1): bf16 KV (the credited format) vs fp8 KV
# (labelled variant), A/B/A on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4u
for kv in bf16 fp8 bf16; do
  timeout -k 10 420 python tools/bench_aggregator.py --kv-dtype $kv > gpurun_out/r4u/agg_$kv.json \
    2> gpurun_out/r4u/agg_$kv.err || { tail -5 gpurun_out/r4u/agg_$kv.err; exit 1; }
  cat gpurun_out/r4u/agg_$kv.json | tee -a gpurun_out/r4u/agg_kv_ab.jsonl
done
