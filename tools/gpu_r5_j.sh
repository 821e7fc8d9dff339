#!/bin/bash
# round 5: the o projection merging the attention splits (one row of a TP shard), 8-wave register-streaming
# workgroups for one row, TP-shard attention up to 128 splits: kernel tests, then whole-step A/Bs in situ (one
# engine per shape, variants interleaved)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode or skinny or fp8 or resid or consumer_merge or waves" > gpurun_out/r5_j_tests.txt 2>&1 || exit $?
OUT=gpurun_out/r5_j_insitu.jsonl
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 4000 --variants plan,cmerge:0 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 13500 --variants plan,cmerge:1000000 >> $OUT 2>/dev/null || exit $?
timeout -k 10 500 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,attnsep96,resid:o=skinny,resid:down=skinny >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 10 --ctx 4000 --new 128 --variants plan,resid:o=skinny,resid:down=skinny >> $OUT 2>/dev/null || exit $?
cat $OUT
