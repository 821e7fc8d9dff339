#!/bin/bash
# round 5: config 5's decode (Llama-3-70B fp8, TP=1, B=1, 32k): gate_up + SwiGLU (82.5 us for 470 MB) and qkv
# (18.6 us for 84 MB) on the LDS-DMA fp8 stream kernel instead of the register-streaming one, in situ
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_aa_70b_fp8stream.jsonl
timeout -k 10 900 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --batch 1 --ctx 32000 --new 96 \
  --variants plan,fp8stream:57344:8192:7:1,fp8stream:57344:8192:8:1,fp8stream:10240:8192:5:4,fp8stream:10240:8192:8:4 >> $OUT 2>/dev/null || exit $?
cat $OUT
