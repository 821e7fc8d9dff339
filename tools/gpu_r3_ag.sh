#!/bin/bash
# Prefill attention with a 1-D item-major grid (global heaviest-first order, one kv head per XCD) vs the
# (items, Hkv) grid (.ab_old), then the 2-rank bench rehearsal.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ag
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py -k "prefill or long" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ag/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3ag/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag base) >> gpurun_out/r3ag/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag prologue >> gpurun_out/r3ag/ab.jsonl || exit 1
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag base --hq 64 --hkv 8 --cases 1x32768) >> gpurun_out/r3ag/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag prologue --hq 64 --hkv 8 --cases 1x32768 >> gpurun_out/r3ag/ab.jsonl || exit 1
  (cd .ab_old && timeout -k 10 200 python ../tools/bench_attn_prefill.py --tag base --hq 64 --hkv 8 --cases 1x4096,4x4096 --prefix 28672) >> gpurun_out/r3ag/ab.jsonl || exit 1
  timeout -k 10 200 python tools/bench_attn_prefill.py --tag prologue --hq 64 --hkv 8 --cases 1x4096,4x4096 --prefix 28672 >> gpurun_out/r3ag/ab.jsonl || exit 1
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r3ag/ab.jsonl"):
    r = json.loads(l); d[(r["kind"], r["hq"], r["nseq"], r["L"], r.get("prefix", 0), r["tree"])].append(r["TFLOPs"])
for k in sorted(d): print(k, d[k])
PY
