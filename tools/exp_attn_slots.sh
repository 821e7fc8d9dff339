#!/bin/bash
# Decode-step A/B of the attention split policy (MRSUM_ATTN_SLOTS, MRSUM_ATTN_PPS) at B = 1 / 10 / 39.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for cfg in ${CFGS:-"768 2" "1024 2" "512 2" "768 1"}; do
  set -- $cfg
  MRSUM_ATTN_SLOTS=$1 MRSUM_ATTN_PPS=$2 timeout -k 10 300 python tools/bench_decode.py --batches ${BATCHES:-1,10,39} --new 128 \
    | sed "s/^{/{\"slots\": $1, \"pps\": $2, /" || exit $?
done
