#!/bin/bash
# Persistent decode layer: kernel test (bounded: a seam wait that never completes sets an error word).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/dl
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "persistent_decode_layer" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dl/t.log 2>&1
rc=$?; tail -25 gpurun_out/dl/t.log; exit $rc
