#!/bin/bash
# round 5: TP=8 parity (bf16 8B and fp8 70B geometry, 8 ranks on one GPU), in-situ attention split plans on
# the two-register-set kernel, then the TP=8 shard decomposition (gpu_r5_c.sh)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -s -q --timeout 900 --timeout-method thread \
  "tests/test_tp_parity_gpu.py::test_tp_paths_match_fp32[8-llama3-8b-bf16]" \
  "tests/test_tp_parity_gpu.py::test_tp_paths_match_fp32[8-llama3-70b-fp8]" > gpurun_out/r5_tp8_parity.txt 2>&1
rc=$?
echo "tp8 parity rc=$rc" >> gpurun_out/r5_tp8_parity.txt
if [ $rc -gt 1 ]; then exit $rc; fi
OUT=gpurun_out/r5_attn_plans.jsonl
timeout -k 10 400 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,attnsep48,attnsep64 >> $OUT 2>/dev/null || exit $?
timeout -k 10 400 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --tp-shard 8 --batch 1 --ctx 32000 --new 128 --variants plan,attnsep32 >> $OUT 2>/dev/null || exit $?
bash tools/gpu_r5_c.sh > gpurun_out/r5_c.log 2>&1 || exit $?
echo done
