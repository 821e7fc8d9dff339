#!/bin/bash
# 32x32-MFMA prefill GEMM: numerics vs fp32, then interleaved A/B against the 16x16 tiles; GEMM GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/m32
timeout -k 10 400 python -u tools/exp_gemm_m32.py > gpurun_out/m32/ab.jsonl 2> gpurun_out/m32/ab.err
rc=$?; tail -3 gpurun_out/m32/ab.err; grep -c '"ok": true' gpurun_out/m32/ab.jsonl; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/m32/ab.jsonl") if l.startswith("{") and "variant" in l]
by = {}
for r in rows:
    by.setdefault((r["model"], r["role"], r["M"], r["fp8"]), {})[r["variant"]] = r["tflops_med"]
for k, v in by.items():
    print(k, v, "m32/m16 = %.3f" % (v["m32g4"] / v["m16g4"]))
PY
