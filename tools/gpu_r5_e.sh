#!/bin/bash
# round 5: same-box A/B of the four-register-set decode attention (in-tree build) against the same sources
# with the two-set kernel only (_native/libmrsum_kernels_nodeep.so, tools/build_ab.py): B=1 at 13.5k (the
# headline's final reduce) and the TP=8 shard at B=1 / 10, 4k; alternating builds
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_attn_deep_ab.jsonl
: > $OUT
for r in 1 2; do
  for so in libmrsum_kernels_nodeep.so libmrsum_kernels.so; do
    SO=$PWD/llm_map_reduce_summarizer_amd/_native/$so
    MRSUM_KERNELS_SO=$SO timeout -k 10 300 python tools/bench_decode.py --batches 1 --ctx 13500 --new 256 2>/dev/null \
      | sed "s|^{|{\"so\": \"$so\", |" >> $OUT || exit 1
    MRSUM_KERNELS_SO=$SO timeout -k 10 300 python tools/bench_decode.py --batches 1,10 --ctx 4000 --new 256 --tp-shard 8 \
      2>/dev/null | sed "s|^{|{\"so\": \"$so\", |" >> $OUT || exit 1
  done
done
cat $OUT
