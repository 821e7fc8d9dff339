#!/bin/bash
# A/B of the decode-attention split policy (hip.decode_attn_plan knobs MRSUM_ATTN_PPS = pages per split,
# MRSUM_ATTN_FUSED_MAX = split cap of the fused last-arriver merge) on full decode steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out/attn_splits.jsonl; : > $OUT
for V in "4 16" "2 32" "1 64" "2 24"; do
  set -- $V
  for CB in "4000 1" "4000 10" "10000 1" "4000 39"; do
    set -- $V $CB
    echo "pps=$1 fmax=$2 ctx=$3 B=$4"
    MRSUM_ATTN_PPS=$1 MRSUM_ATTN_FUSED_MAX=$2 timeout -k 10 120 python tools/bench_decode.py --ctx $3 --batches $4 --new 256 \
      2>/dev/null | grep "^{" | sed "s/^{/{\"pps\": $1, \"fmax\": $2, /" >> $OUT || exit $?
  done
done
cat $OUT
