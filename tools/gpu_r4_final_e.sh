#!/bin/bash
# Round 4 final tree after the tall-tile stream GEMM: full GPU suite, smoke(), headline at 20 timed steps,
# 24 h single-pass Llama-3.1 reduce.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4final4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4final4/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4final4/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final4/smoke.log 2>&1 || { tail -20 gpurun_out/r4final4/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 python bench.py --steps 20 --warmup 1 > gpurun_out/r4final4/bench20.json 2> gpurun_out/r4final4/bench20.err \
  || { tail -5 gpurun_out/r4final4/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4final4/bench20.json')); print('bench20', d['ms_per_step'], d['value'], d['phases_s'], d['timed_work'])"
timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 --model llama3.1-8b --no-hierarchical \
  > gpurun_out/r4final4/bench24h_single.json 2> gpurun_out/r4final4/bench24h_single.err || { tail -5 gpurun_out/r4final4/bench24h_single.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4final4/bench24h_single.json')); print('24h single-pass', d['ms_per_step'], d['value'], d['timed_work']['pinned_ok'], d['phases_s'])"
