#!/bin/bash
# Decode steps for the planner fit: TP=1 and one rank's TP=2/4/8 shard (TP push + one-rank all-reduce
# emulation), B = 1/5/10/20/39 at 4k context, two rounds.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3n
OUT=gpurun_out/r3n/steps.jsonl
: > $OUT
for round in 0 1; do
  for tp in 1 2 4 8; do
    timeout -k 10 300 python tools/bench_decode.py --tp-shard $tp --batches 1,5,10,20,39 --new 192 \
      2>/dev/null | sed "s/^{/{\"round\": $round, /" >> $OUT || exit 1
  done
done
cat $OUT
timeout -k 10 300 python -u -m pytest tests/test_custom_ar_gpu.py -x -v -s --timeout 280 --timeout-method thread \
  -p no:cacheprovider -k "two_ranks" > gpurun_out/r3n/ar.log 2>&1
rc=$?; grep -h "fused all-reduce cost" gpurun_out/r3n/ar.log; exit $rc
