#!/bin/bash
# round 5: full GPU test suite, then a short headline bench (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread \
    > gpurun_out/r5_gpu_tests.txt 2>&1
rc=$?
echo "gpu tests rc=$rc" >> gpurun_out/r5_gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 > gpurun_out/r5_bench_quick.json 2> gpurun_out/r5_bench_quick.err
echo "bench rc=$?"
exit $rc
