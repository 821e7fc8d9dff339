#!/bin/bash
# Same-box A/B of the prefill GEMM between two kernel-library builds (MRSUM_KERNELS_SO): the in-tree build vs
# _native/libmrsum_kernels_${BASE}.so, alternating processes, tools/bench_gemm.py (8B bf16 + 70B fp8 gate_up).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/gemmab
OUT=gpurun_out/gemmab/${BASE}.jsonl
: > $OUT
for r in 1 2 3; do
  for so in llm_map_reduce_summarizer_amd/_native/libmrsum_kernels.so llm_map_reduce_summarizer_amd/_native/libmrsum_kernels_${BASE}.so; do
    MRSUM_KERNELS_SO=$PWD/$so timeout -k 10 200 python tools/bench_gemm.py --ms 4096,16384 --variants g4 --rounds 5 2>/dev/null \
      | sed "s|^{|{\"so\": \"$(basename $so)\", \"rep\": $r, |" >> $OUT || exit 1
  done
done
python - "$OUT" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    by[(r["role"], r["M"])][r["so"]].append(r["tflops_med"])
for k, v in by.items():
    a, b = [sorted(x)[len(x) // 2] for x in v.values()]
    print(k, {s: sorted(x) for s, x in v.items()}, "alt/base = %.3f" % (b / a))
PY
