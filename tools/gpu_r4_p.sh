#!/bin/bash
# Round 4: headline bench after the class-1 attention plan change (3 timed steps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4p
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/r4p/bench.json 2> gpurun_out/r4p/bench.err \
  || { tail -5 gpurun_out/r4p/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4p/bench.json')); print('bench', d['ms_per_step'], d['value'], d['phases_s'], d['reduce_plan'], d['timed_work'])"
