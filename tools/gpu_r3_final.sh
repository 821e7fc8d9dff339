#!/bin/bash
# Final-tree verification: full GPU suite, smoke(), headline bench (3 timed steps), BASELINE config 5, and a
# rocprofv3 kernel split of one bench step.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/final/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
echo smoke ok
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -5 gpurun_out/final/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print('bench', d['ms_per_step'], d['value'], d['engine_rank0']['prefill_tok_s'])"
timeout -k 10 400 python tools/bench_aggregator.py > gpurun_out/final/agg70.json 2> gpurun_out/final/agg70.err || { tail -5 gpurun_out/final/agg70.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/agg70.json')); print('config5', d['value'], d['prefill_s'], d['decode_ms_per_token'])"
NAME=final/prof TO=400 bash tools/gpu_prof.sh || exit 1
head -24 gpurun_out/final/prof/summary.txt
