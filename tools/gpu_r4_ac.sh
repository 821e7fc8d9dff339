#!/bin/bash
# Tall-tile stream GEMM (65-128 decode rows in one pass over the weights) vs the 64-row chunks, on the
# 24 h transcript (map batch 92 in graph bucket 96): stream GEMM tests, then bench A/B/A/B on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4ac
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stream_gemm" -p no:cacheprovider > gpurun_out/r4ac/tests.log 2>&1 || { tail -20 gpurun_out/r4ac/tests.log; exit 1; }
tail -1 gpurun_out/r4ac/tests.log
for r in 1 2; do
  for t in 128 64; do
    MRSUM_STREAM_TALL_M=$t timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 > gpurun_out/r4ac/b_$t.json \
      2> gpurun_out/r4ac/b_$t.err || { tail -5 gpurun_out/r4ac/b_$t.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4ac/b_$t.json')); print(json.dumps({'stream_tall_m': $t, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'phases_s': d['phases_s'], 'pinned_ok': d['timed_work']['pinned_ok'], 'decode_s': d['engine_rank0']['decode_s']}))" | tee -a gpurun_out/r4ac/ab.jsonl
  done
done
