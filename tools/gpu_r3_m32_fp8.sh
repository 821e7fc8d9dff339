#!/bin/bash
# 32x32 vs 16x16 MFMA tiles on the 70B fp8 prefill GEMMs over several M (second look at gate_up + SwiGLU).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/m32fp8
timeout -k 10 400 python -u tools/exp_gemm_m32.py --skip-check --skip-bf16 --fp8-ms 4096,8192,16384,32768 --rounds 7 \
  > gpurun_out/m32fp8/ab.jsonl 2> gpurun_out/m32fp8/ab.err
rc=$?; tail -3 gpurun_out/m32fp8/ab.err; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/m32fp8/ab.jsonl") if l.startswith("{") and "variant" in l]
by = {}
for r in rows:
    by.setdefault((r["role"], r["M"]), {})[r["variant"]] = r["tflops_med"]
for k, v in by.items():
    print(k, v, "m32/m16 = %.3f" % (v["m32g4"] / v["m16g4"]))
PY
