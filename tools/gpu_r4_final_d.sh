#!/bin/bash
# Round 4 final tree (end of session: probe kernels, blas knob): full GPU suite, smoke(), headline bench at 20 timed steps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4final3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4final3/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4final3/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final3/smoke.log 2>&1 || { tail -20 gpurun_out/r4final3/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 700 python bench.py --steps 20 --warmup 1 > gpurun_out/r4final3/bench20.json 2> gpurun_out/r4final3/bench20.err \
  || { tail -5 gpurun_out/r4final3/bench20.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4final3/bench20.json')); print('bench20', d['ms_per_step'], d['value'], d['phases_s'], d['timed_work'])"
