#!/bin/bash
# Headline bench (3 timed steps), BASELINE config 5 (70B fp8 aggregator pass at 32k), then a rocprofv3
# kernel-trace of one bench step.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3x
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/r3x/bench.json 2> gpurun_out/r3x/bench.err \
  || { tail -5 gpurun_out/r3x/bench.err; exit 1; }
cat gpurun_out/r3x/bench.json
timeout -k 10 400 python tools/bench_aggregator.py > gpurun_out/r3x/agg70.json 2> gpurun_out/r3x/agg70.err \
  || { tail -5 gpurun_out/r3x/agg70.err; exit 1; }
cat gpurun_out/r3x/agg70.json
NAME=r3x/prof TO=400 bash tools/gpu_prof.sh || exit 1
head -30 gpurun_out/r3x/prof/summary.txt
