#!/bin/bash
# round 5: full GPU test suite on the current tree, then BASELINE config 5 (Llama-3-70B fp8 aggregator pass,
# 32k context, 1000 pinned tokens, TP=1): bf16 KV (credited) and the fp8v KV variant (labelled)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 600 --timeout-method thread \
    > gpurun_out/r5_l_gpu_tests.txt 2>&1
rc=$?
echo "gpu tests rc=$rc" >> gpurun_out/r5_l_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u tools/bench_aggregator.py --steps 1 --warmup 1 > gpurun_out/r5_l_config5.jsonl 2> gpurun_out/r5_l_config5.err || exit $?
timeout -k 10 240 python -u tools/bench_aggregator.py --steps 1 --warmup 1 --kv-dtype fp8v >> gpurun_out/r5_l_config5.jsonl 2>> gpurun_out/r5_l_config5.err || exit $?
exit $rc
