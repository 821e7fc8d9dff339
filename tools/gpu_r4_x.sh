#!/bin/bash
# Weight-tile read order vs HBM bandwidth (tools/exp_row_pattern.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4x
timeout -k 10 300 python tools/exp_row_pattern.py > gpurun_out/r4x/row_pattern.jsonl 2> gpurun_out/r4x/row_pattern.err \
  || { tail -5 gpurun_out/r4x/row_pattern.err; exit 1; }
cat gpurun_out/r4x/row_pattern.jsonl
