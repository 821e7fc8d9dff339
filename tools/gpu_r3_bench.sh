#!/bin/bash
# Headline bench (driver config, fewer steps) + smoke.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/bench
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/bench/smoke.log 2>&1 || { tail -5 gpurun_out/bench/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err || { tail -5 gpurun_out/bench/bench.err; exit 1; }
cat gpurun_out/bench/bench.json
