#!/bin/bash
# TP push (row-parallel decode GEMM all-reducing its own tiles): kernel + 2-rank tests, then TP-shard decode
# steps: push with the register-streaming producer (auto), push with the stream producer, no push.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3k
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py -x -v --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "tp_push or tp2 or skinny_resid" > gpurun_out/r3k/tests.log 2>&1
rc=$?; tail -8 gpurun_out/r3k/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r3k/steps.jsonl
: > $OUT
for tp in 8 4 2; do
  for v in "1 auto" "1 stream" "0 auto"; do
    set -- $v
    MRSUM_TP_PUSH=$1 MRSUM_TP_RESID_KERNEL=$2 timeout -k 10 300 python tools/bench_decode.py --tp-shard $tp \
      --batches 1,10,16 --new 192 2>/dev/null | sed "s/^{/{\"push\": $1, \"resid\": \"$2\", /" >> $OUT || exit 1
  done
done
cat $OUT
