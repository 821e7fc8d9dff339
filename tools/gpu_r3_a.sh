#!/bin/bash
# Round 3: interleaved-prefill GPU test, then TP=1 / TP=8-shard decode steps and a TP=8-shard kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/base
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -k "interleaved or native" > gpurun_out/base/inter_test.log 2>&1
rc=$?; tail -4 gpurun_out/base/inter_test.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_base_decode.sh
