#!/bin/bash
# round 5: parity numbers (printed), the 8-rank TP parity tests with per-rank diagnostics, then the
# K/V prefetch and KV-format decode experiments (tools/gpu_r5_b.sh)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -s -q --timeout 300 --timeout-method thread \
  tests/test_forward_parity_gpu.py tests/test_kernels_gpu.py::test_rope_kv_fp8_cache_tiny_rows \
  > gpurun_out/r5_parity.txt 2>&1
echo "parity rc=$?" >> gpurun_out/r5_parity.txt
timeout -k 10 900 python -u -m pytest -s -q --timeout 880 --timeout-method thread tests/test_tp_parity_gpu.py \
  > gpurun_out/r5_tp_parity.txt 2>&1
rc=$?
echo "tp parity rc=$rc" >> gpurun_out/r5_tp_parity.txt
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_r5_b.sh
