#!/bin/bash
# round 5: TP=8 parity on one shared GPU with the self-test's per-path reasons, then the four-register-set
# attention A/B (gpu_r5_e.sh) and the in-situ attention plans (gpu_r5_f.sh)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -s -q --timeout 880 --timeout-method thread \
  "tests/test_tp_parity_gpu.py::test_tp_paths_match_fp32[8-llama3-8b-bf16]" > gpurun_out/r5_tp8_parity_diag.txt 2>&1
rc=$?
echo "tp8 parity rc=$rc" >> gpurun_out/r5_tp8_parity_diag.txt
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_r5_e.sh > gpurun_out/r5_e.log 2>&1 || exit $?
bash tools/gpu_r5_f.sh > gpurun_out/r5_f.log 2>&1 || exit $?
echo done
