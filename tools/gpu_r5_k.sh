#!/bin/bash
# round 5: fp8 register-streaming TP-push producers (70B fp8 TP=8 shard o / down), consumer merge removed:
# kernel tests, the custom all-reduce / TP parity tests (self-test of every push path incl. fp8 skinny at the
# 70B shard shapes), then in-situ A/Bs of the new producer rule
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode or attn_prefill or skinny or fp8 or resid or waves" > gpurun_out/r5_k_tests.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -q -x --timeout 900 --timeout-method thread tests/test_custom_ar_gpu.py \
  "tests/test_tp_parity_gpu.py::test_tp_paths_match_fp32[8-llama3-70b-fp8]" -s > gpurun_out/r5_k_tp_tests.txt 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attn_prefill.py --qb 1,2,1,2 --cases 8x4096,39x4000,1x32768 > gpurun_out/r5_k_attn_prefill_qb.jsonl 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attn_prefill.py --qb 1,2,1,2 --hq 64 --hkv 8 --cases 1x32768,4x8192 >> gpurun_out/r5_k_attn_prefill_qb.jsonl 2>&1 || exit $?
OUT=gpurun_out/r5_k_insitu.jsonl
timeout -k 10 500 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,resid:o=stream,resid:down=stream >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 10 --ctx 4000 --new 128 --variants plan,resid:o=stream >> $OUT 2>/dev/null || exit $?
cat $OUT
OUT2=gpurun_out/r5_k_70b_tp1.jsonl
timeout -k 10 600 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --batch 1 --ctx 32000 --new 96 --variants plan,attnsep48,attnsep64,waves:8 >> $OUT2 2>/dev/null || exit $?
cat $OUT2
