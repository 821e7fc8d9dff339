#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_forward_parity_gpu.py -x -v -s --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "fp8" > gpurun_out/r3e/tests.log 2>&1
rc=$?; grep -E "parity:|passed|failed" gpurun_out/r3e/tests.log | tail -6
TAG=sc1 bash tools/gpu_ab_so.sh || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8 -o run -- python3 tools/bench_decode.py --batches 1 --new 128 --tp-shard 8 > gpurun_out/r3e/p8.log 2>&1 || exit $?
python3 tools/trace_summary.py /tmp/p8 > gpurun_out/r3e/p8_summary.txt 2>&1
python3 tools/trace_gaps.py /tmp/p8 > gpurun_out/r3e/p8_gaps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p1 -o run -- python3 tools/bench_decode.py --batches 1 --new 128 > gpurun_out/r3e/p1.log 2>&1 || exit $?
python3 tools/trace_summary.py /tmp/p1 > gpurun_out/r3e/p1_summary.txt 2>&1
python3 tools/trace_gaps.py /tmp/p1 > gpurun_out/r3e/p1_gaps.txt 2>&1
head -25 gpurun_out/r3e/p8_summary.txt
exit $rc
