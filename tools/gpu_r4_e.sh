#!/bin/bash
# Config 5 (Llama-3-70B fp8 aggregator, 32k context, TP=1): two-term fp8 QKV input on / off (A/B on one box), plus
# the fp8 / fp8-KV parity tests and the fp8-KV B = 10 split plan in situ.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4e
timeout -k 10 300 python -u -m pytest tests/test_forward_parity_gpu.py -m gpu -x -q -s --timeout 240 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4e/parity.log 2>&1 || { tail -20 gpurun_out/r4e/parity.log; exit 1; }
grep -E "parity" gpurun_out/r4e/parity.log
for split in 1 0 1; do
  MRSUM_FP8_QKV_SPLIT=$split timeout -k 10 420 python tools/bench_aggregator.py > gpurun_out/r4e/agg_split$split.json \
    2> gpurun_out/r4e/agg_split$split.err || { tail -5 gpurun_out/r4e/agg_split$split.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4e/agg_split$split.json')); d['fp8_qkv_split']=$split; print(json.dumps(d))" | tee -a gpurun_out/r4e/agg_ab.jsonl
done
