#!/bin/bash
# fp8 stream GEMM with 16-B A reads (no merged ds_read2st64 -> no vmcnt(0) drain per slot): fp8 kernel tests,
# then the 70B decode GEMM sweep on the base (.ab_old) and this tree, then the 70B fp8 decode step at 32k.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ab
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_forward_parity_gpu.py -k "fp8" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3ab/tests.log; [ $rc -eq 0 ] || exit $rc
(cd .ab_old && timeout -k 10 300 python ../tools/sweep_fp8_decode.py --ms 1,8) > gpurun_out/r3ab/base.jsonl 2> gpurun_out/r3ab/base.err || exit 1
timeout -k 10 300 python tools/sweep_fp8_decode.py --ms 1,8 > gpurun_out/r3ab/new.jsonl 2> gpurun_out/r3ab/new.err || exit 1
python - <<'PY'
import json
def best(f):
    b = {}
    for l in open(f):
        if not l.startswith("{"): continue
        r = json.loads(l); k = (r["op"], r["M"], r["kind"])
        if k not in b or r["us"] < b[k]["us"]: b[k] = r
    return b
a, n = best("gpurun_out/r3ab/base.jsonl"), best("gpurun_out/r3ab/new.jsonl")
for k in sorted(a):
    if k[2] == "stream": print(k, "base", a[k]["cfg"], a[k]["us"], a[k]["TBps"], "| new", n[k]["cfg"], n[k]["us"], n[k]["TBps"])
PY
timeout -k 10 400 python3 tools/bench_decode.py --model llama3-70b --dtype fp8 --ctx 32000 --batches 1 --new 48 > gpurun_out/r3ab/d70.log 2>&1 || exit 1
grep "^{" gpurun_out/r3ab/d70.log
