#!/bin/bash
# round 5: ping-pong decode attention (two LDS tile buffers, one barrier per tile) on grids of <= 512 workgroups:
# kernel tests, then whole-step A/Bs in situ against the single-buffer kernel (pp:0)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn_decode" > gpurun_out/r5_u_tests.txt 2>&1 || exit $?
OUT=gpurun_out/r5_u_pp_insitu.jsonl
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,pp:0 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 10 --ctx 6000 --variants plan,pp:0 >> $OUT 2>/dev/null || exit $?
timeout -k 10 300 python tools/exp_plans_insitu.py --tp-shard 8 --batch 1 --ctx 4000 --variants plan,pp:0 >> $OUT 2>/dev/null || exit $?
timeout -k 10 500 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --batch 1 --ctx 32000 --new 96 --variants plan,pp:0 >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,pp:0 >> $OUT 2>/dev/null || exit $?
cat $OUT
