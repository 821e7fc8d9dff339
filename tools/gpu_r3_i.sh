#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3i/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3i/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/p70 -o run -- python3 tools/bench_decode.py --model llama3-70b --dtype fp8 --batches 1 --ctx 32000 --new 64 > gpurun_out/r3i/p70.log 2>&1 || exit $?
python3 tools/trace_summary.py /tmp/p70 > gpurun_out/r3i/p70_summary.txt 2>&1
python3 tools/trace_gaps.py /tmp/p70 > gpurun_out/r3i/p70_gaps.txt 2>&1
head -30 gpurun_out/r3i/p70_gaps.txt
