#!/bin/bash
# Driver-length headline bench (20 timed steps, 1 warmup) on the restored tree.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/bench20
timeout -k 10 1000 python bench.py --steps 20 --warmup 1 > gpurun_out/bench20/bench.json 2> gpurun_out/bench20/bench.err || { tail -5 gpurun_out/bench20/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench20/bench.json')); print('bench', d['ms_per_step'], d['value'], d['engine_rank0']['prefill_tok_s'], d['phases_s'])"
