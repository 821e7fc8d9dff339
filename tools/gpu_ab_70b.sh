#!/bin/bash
# Same-box A/B of the Llama-3-70B fp8 decode step (B=1, CTX context): .ab_old (a git worktree of an earlier
# commit, built in-tree) vs this tree, alternating twice; then, with AGG=1, the BASELINE config-5
# aggregator pass (32k context, 1000 new tokens) on this tree.  GPU tests first (TESTS=pytest -k filter).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "$TESTS" > gpurun_out/ab70_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/ab70_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --model llama3-70b --dtype fp8 --batches "${BATCHES:-1}" \
      --ctx "${CTX:-8000}" --new 128 | sed "s|^{|{\"tree\": \"$t\", |") || exit 1
  done
done
if [ "${AGG:-0}" = 1 ]; then
  timeout -k 10 400 python tools/bench_aggregator.py || exit 1
fi
