#!/bin/bash
# fp8 decode GEMMs at 70B shapes: the real kernels vs a build whose fp8 -> bf16 conversion is a bit-cast
# (wrong numbers, same memory traffic): is the W8A16 stream conversion-bound?
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3y
timeout -k 10 300 python tools/sweep_fp8_decode.py --ms 1,8 > gpurun_out/r3y/cvt.jsonl 2> gpurun_out/r3y/cvt.err || { tail -3 gpurun_out/r3y/cvt.err; exit 1; }
MRSUM_KERNELS_SO=$PWD/llm_map_reduce_summarizer_amd/_native/libmrsum_kernels_nocvt.so timeout -k 10 300 \
  python tools/sweep_fp8_decode.py --ms 1,8 > gpurun_out/r3y/nocvt.jsonl 2> gpurun_out/r3y/nocvt.err || { tail -3 gpurun_out/r3y/nocvt.err; exit 1; }
python - <<'PY'
import json
def best(f):
    b = {}
    for l in open(f):
        if not l.startswith("{"): continue
        r = json.loads(l); k = (r["op"], r["M"], r["kind"])
        if k not in b or r["us"] < b[k]["us"]: b[k] = r
    return b
a, n = best("gpurun_out/r3y/cvt.jsonl"), best("gpurun_out/r3y/nocvt.jsonl")
for k in sorted(a):
    print(k, "cvt", a[k]["cfg"], a[k]["us"], a[k]["TBps"], "| nocvt", n[k]["cfg"], n[k]["us"], n[k]["TBps"])
PY
