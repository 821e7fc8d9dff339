#!/bin/bash
# round 5, final engine (pinned windows, one-sync admission): BASELINE config 5, two timed passes
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_aggregator.py --steps 2 --warmup 1 > gpurun_out/r5_kk_config5.jsonl 2> gpurun_out/r5_kk_config5.err
rc=$?; echo "rc=$rc"; tail -n 2 gpurun_out/r5_kk_config5.jsonl | cut -c1-300; exit $rc
