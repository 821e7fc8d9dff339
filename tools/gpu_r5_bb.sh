#!/bin/bash
# round 5 final tree: the headline bench at the driver's length (20 timed steps, 5 warmup)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_20steps_final.json 2> gpurun_out/r5_bench_20steps_final.err
rc=$?
tail -n 1 gpurun_out/r5_bench_20steps_final.json
exit $rc
