#!/bin/bash
# Round 3: the whole GPU test suite (new: interleaved prefill, forward parity, sc1 last-arriver loads), then
# the same-box decode A/B of the previous kernel library vs this tree.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3b
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r3b/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3b/gpu_tests.log; grep -E "parity|passed|failed" gpurun_out/r3b/gpu_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc

