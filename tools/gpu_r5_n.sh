#!/bin/bash
# round 5: the fp8 register-streaming kernel issuing its first weight block before staging the x slice in
# LDS (skinny_gemm.hip skinny_fp8_kernel XL): kernel tests, then a same-box A/B of the two library builds
# (_native/libmrsum_kernels_base.so = before) on Llama-3-70B fp8 decode at 32k: TP=1 (config 5) and the TP=8 shard
set -uo pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8" > gpurun_out/r5_n_tests.txt 2>&1 || exit $?
OUT=gpurun_out/r5_n_xl_prologue_ab.jsonl
: > $OUT
for r in 1 2; do
  for so in llm_map_reduce_summarizer_amd/_native/libmrsum_kernels_base.so llm_map_reduce_summarizer_amd/_native/libmrsum_kernels.so; do
    for tp in 1 8; do
      MRSUM_KERNELS_SO=$PWD/$so timeout -k 10 300 python tools/bench_decode.py --model llama3-70b --dtype fp8 --batches 1 \
        --ctx 32000 --new 96 --tp-shard $tp 2>/dev/null | sed "s|^{|{\"so\": \"$(basename $so)\", |" >> $OUT || exit 1
    done
  done
done
cat $OUT
