#!/bin/bash
# The decode LM head of 65-128 rows on the tall-tile stream GEMM (MRSUM_LINEAR_TALL=1) vs the 256 x 256-tile
# GEMM (=0), 24 h transcript, A/B/A/B on one box; then the tall-tile tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4ad
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stream_gemm or linear" -p no:cacheprovider > gpurun_out/r4ad/tests.log 2>&1 || { tail -20 gpurun_out/r4ad/tests.log; exit 1; }
tail -1 gpurun_out/r4ad/tests.log
for r in 1 2; do
  for t in 1 0; do
    MRSUM_LINEAR_TALL=$t timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 > gpurun_out/r4ad/b_$t.json \
      2> gpurun_out/r4ad/b_$t.err || { tail -5 gpurun_out/r4ad/b_$t.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4ad/b_$t.json')); print(json.dumps({'linear_tall': $t, 'round': $r, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'phases_s': d['phases_s'], 'pinned_ok': d['timed_work']['pinned_ok'], 'decode_s': d['engine_rank0']['decode_s']}))" | tee -a gpurun_out/r4ad/ab.jsonl
  done
done
