#!/bin/bash
# Iteration script (deferred-norm decode work): stream-GEMM kernel tests, decode-step bench, B=1 attention sweep.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/dn
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "deferred_norm or stream_gemm or stream_fp8 or swiglu_split or tp_shard_decode" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dn/k.log 2>&1
rc=$?; tail -2 gpurun_out/dn/k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_decode.py --batches 1,10,39 > gpurun_out/dn/dec.log 2>&1
rc=$?; grep "^{" gpurun_out/dn/dec.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${ATTN_SWEEP:-}" ]; then
timeout -k 10 300 python -u tools/bench_attn_decode.py --batches 1 --ctx ${ATTN_CTX:-4000} --splits auto,8,16,24,32,48 > gpurun_out/dn/attn.log 2>&1
rc=$?; grep "^{" gpurun_out/dn/attn.log; exit $rc
fi
