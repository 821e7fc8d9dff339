#!/bin/bash
# Round-3 tree: BASELINE's 24 h configs (2-level reduce on llama3-8b; single-pass reduce on llama3.1-8b).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3aj
timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 > gpurun_out/r3aj/b24.json 2> gpurun_out/r3aj/b24.err || { tail -3 gpurun_out/r3aj/b24.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3aj/b24.json')); print('24h', d['ms_per_step'], d['value'], d['reduce_plan'])"
timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 --model llama3.1-8b --no-hierarchical > gpurun_out/r3aj/b24sp.json 2> gpurun_out/r3aj/b24sp.err || { tail -3 gpurun_out/r3aj/b24sp.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3aj/b24sp.json')); print('24h single pass', d['ms_per_step'], d['value'], d['reduce_plan'])"
