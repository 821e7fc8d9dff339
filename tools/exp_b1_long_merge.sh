#!/bin/bash
# A/B of the split merge for one sequence at ~10k context (the final reduce's decode): default
# (64 splits, separate merge kernel), fused merge capped at 32 splits, fused merge over 64 splits.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/b1_long_merge.jsonl; : > $OUT
for R in 1 2; do
  for V in "auto 32" "1 32" "1 64"; do
    set -- $V
    MRSUM_FUSED_COMBINE=$1 MRSUM_ATTN_FUSED_MAX=$2 timeout -k 10 120 python tools/bench_decode.py --ctx 10000 --batches 1 --new 256 \
      2>/dev/null | grep "^{" | sed "s/^{/{\"fused_combine\": \"$1\", \"fused_max\": $2, /" >> $OUT || exit $?
  done
done
cat $OUT
