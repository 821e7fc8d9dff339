#!/bin/bash
# Same-box A/B of two kernel-library builds (MRSUM_KERNELS_SO): _native/libmrsum_kernels_${BASE:-base}.so vs
# the in-tree build, alternating, decode steps at 4k context for TP=1 and the TP=8 shard (tools/bench_decode.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/ab
OUT=gpurun_out/ab/${TAG:-ab}.jsonl
: > $OUT
for r in ${REPS:-1 2}; do
  for so in llm_map_reduce_summarizer_amd/_native/libmrsum_kernels_${BASE:-base}.so llm_map_reduce_summarizer_amd/_native/libmrsum_kernels.so; do
    for tp in ${TPS:-1 8}; do
      MRSUM_KERNELS_SO=$PWD/$so timeout -k 10 300 python tools/bench_decode.py --batches ${BATCHES:-1,10,39} --ctx 4000 \
        --new 256 --tp-shard $tp 2>/dev/null | sed "s|^{|{\"so\": \"$(basename $so)\", |" >> $OUT || exit 1
    done
  done
done
cat $OUT
