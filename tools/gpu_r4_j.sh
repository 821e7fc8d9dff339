#!/bin/bash
# Round 4: four-wave bf16 GEMM -- correctness, then rates against gemm.hip and hipBLASLt.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4j
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k gemm4w --timeout 120 --timeout-method thread \
  > gpurun_out/r4j/test.log 2>&1 || { tail -30 gpurun_out/r4j/test.log; exit 1; }
tail -2 gpurun_out/r4j/test.log
timeout -k 10 300 python tools/bench_gemm4w.py > gpurun_out/r4j/bench.jsonl 2> gpurun_out/r4j/bench.err \
  || { tail -20 gpurun_out/r4j/bench.err; exit 1; }
cat gpurun_out/r4j/bench.jsonl
