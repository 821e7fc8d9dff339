#!/bin/bash
# Headline bench A/B/A on one box: plain prefill GEMMs (qkv, o, down) on gemm.hip (default) vs hipBLASLt
# (MRSUM_GEMM_KERNEL=blas; the SwiGLU gate_up GEMM stays on gemm.hip).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4v
for k in 8w blas 8w blas; do
  MRSUM_GEMM_KERNEL=$k timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/r4v/bench_$k.json \
    2> gpurun_out/r4v/bench_$k.err || { tail -5 gpurun_out/r4v/bench_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4v/bench_$k.json')); print(json.dumps({'gemm_kernel': '$k', 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'phases_s': d['phases_s'], 'engine': d.get('engine_rank0')}))" | tee -a gpurun_out/r4v/ab.jsonl
done
