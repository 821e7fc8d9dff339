#!/bin/bash
# 32x32 vs 16x16 MFMA tiles on the bf16 gate_up + SwiGLU prefill GEMM over M, 9 interleaved rounds (twice).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/m32gu
for rep in 1 2; do
timeout -k 10 300 python -u tools/exp_gemm_m32.py --skip-check --bf16-roles gate_up,qkv,down --ms 4096,8192,16384,32768 --fp8-model "" --rounds 9 \
  > gpurun_out/m32gu/ab$rep.jsonl 2> gpurun_out/m32gu/ab$rep.err
rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/m32gu/ab$rep.err; exit $rc; }
done
python - <<'PY'
import json
for rep in (1, 2):
    rows = [json.loads(l) for l in open("gpurun_out/m32gu/ab%d.jsonl" % rep) if l.startswith("{") and "variant" in l]
    by = {}
    for r in rows:
        by.setdefault((r["role"], r["M"]), {})[r["variant"]] = r["tflops_med"]
    for k, v in by.items():
        print(rep, k, v, "m32/m16 = %.3f" % (v["m32g4"] / v["m16g4"]))
PY
