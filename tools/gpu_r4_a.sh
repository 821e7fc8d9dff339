#!/bin/bash
# Round 4 first check: EOS-at-replay + odd-GQA-ratio GPU tests, smoke (build stamps), headline bench with the
# pinned-work assertion.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_custom_ar_gpu.py tests/test_kernels_gpu.py -k "engine or attn or sampler or eos or gqa or custom or tp2" \
  -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4a/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { tail -5 gpurun_out/r4a/smoke.log; exit 1; }
tail -2 gpurun_out/r4a/smoke.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r4a/bench.err
python -c "import json; d=json.load(open('gpurun_out/r4a/bench.json')); print('bench', d['ms_per_step'], d['value'], d['timed_work'], d['engine_rank0']['prefill_tok_s'])"
exit $rc
