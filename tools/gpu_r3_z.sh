#!/bin/bash
# bf16 stream GEMM at the 70B fp8 decode shapes' row bytes (is the fp8 kernel or the shape slow?)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3z
timeout -k 10 300 python tools/sweep_stream_cfg.py --ms 1 --ops down70h,o70,gate_up,down > gpurun_out/r3z/bf16.jsonl 2> gpurun_out/r3z/bf16.err || { tail -3 gpurun_out/r3z/bf16.err; exit 1; }
python - <<'PY'
import json
b = {}
for l in open("gpurun_out/r3z/bf16.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    if r["op"] not in b or r["us"] < b[r["op"]]["us"]: b[r["op"]] = r
for k, r in b.items(): print(k, r)
PY
