#!/bin/bash
# Round 4 final tree, part B: the headline bench at the driver's length (20 timed steps) and a rocprofv3 kernel
# split of one bench step.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4final
timeout -k 10 700 python bench.py --steps 20 --warmup 1 > gpurun_out/r4final/bench20.json 2> gpurun_out/r4final/bench20.err \
  || { tail -5 gpurun_out/r4final/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4final/bench20.json')); print('bench20', d['ms_per_step'], d['value'], d['timed_work'])"
NAME=r4final/prof TO=400 bash tools/gpu_prof.sh || exit 1
head -30 gpurun_out/r4final/prof/summary.txt
