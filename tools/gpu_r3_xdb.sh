#!/bin/bash
# X0 double-buffered bf16 GEMM (group_m bit 9): numerics vs fp32, then interleaved A/B vs the committed schedule.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/xdb
timeout -k 10 400 python -u tools/exp_gemm_m32.py --variants m16g4=4,xdbg4=516 --ms 4096,16384,32768 --fp8-model "" --rounds 9 \
  > gpurun_out/xdb/ab.jsonl 2> gpurun_out/xdb/ab.err
rc=$?; tail -3 gpurun_out/xdb/ab.err; grep -c '"ok": true' gpurun_out/xdb/ab.jsonl; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/xdb/ab.jsonl") if l.startswith("{") and "variant" in l]
by = {}
for r in rows:
    by.setdefault((r["role"], r["M"]), {})[r["variant"]] = r["tflops_med"]
for k, v in by.items():
    print(k, v, "xdb/m16 = %.3f" % (v["xdbg4"] / v["m16g4"]))
PY
