#!/bin/bash
# A/B: decode-attention split merge fused into the attention launch (MRSUM_FUSED_COMBINE=1) vs the
# auto policy (separate merge kernel above 64 (sequence, kv head) groups) at TP=1 batch sizes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/fused_merge_tp1.jsonl; : > $OUT
for FC in auto 1 auto 1; do
  for CB in "4000 39" "4000 10" "6000 10"; do
    set -- $CB
    echo "fc=$FC ctx=$1 B=$2"
    MRSUM_FUSED_COMBINE=$FC timeout -k 10 120 python tools/bench_decode.py --ctx $1 --batches $2 --new 256 \
      2>/dev/null | grep "^{" | sed "s/^{/{\"fused_combine\": \"$FC\", /" >> $OUT || exit $?
  done
done
cat $OUT
