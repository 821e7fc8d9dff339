#!/bin/bash
# round 5 final tree: full GPU suite, smoke(), config 5 (bf16 KV, credited) and the 10 h headline with the
# fp8v KV variant (labelled, 3 timed steps)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 600 --timeout-method thread \
    > gpurun_out/r5_x_gpu_tests.txt 2>&1
rc=$?
echo "gpu tests rc=$rc" >> gpurun_out/r5_x_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_x_smoke.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/bench_aggregator.py --steps 1 --warmup 1 > gpurun_out/r5_x_config5.jsonl 2> gpurun_out/r5_x_config5.err || exit $?
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --kv-dtype fp8v > gpurun_out/r5_x_bench_fp8v.json 2> gpurun_out/r5_x_bench_fp8v.err || exit $?
timeout -k 10 600 python tools/exp_plans_insitu.py --batch 39 --ctx 4400 --new 128 --variants plan,qkv:stream:6:8,qkv:stream:4:8,qkv:stream:8:16 >> gpurun_out/r5_y_b39_qkv.jsonl 2>/dev/null || exit $?
exit $rc
