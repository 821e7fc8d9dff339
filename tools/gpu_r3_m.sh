#!/bin/bash
# skinny deferred-norm SwiGLU with register-resident norm loads: tests, TP-shard steps (push on/off), B=1 trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3m
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 280 --timeout-method thread \
  -p no:cacheprovider -k "tp_push or skinny_resid or swiglu" > gpurun_out/r3m/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3m/tests.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r3m/steps.jsonl
: > $OUT
for tp in 8 4 2; do
  for push in 1 0; do
    MRSUM_TP_PUSH=$push timeout -k 10 300 python tools/bench_decode.py --tp-shard $tp --batches 1,10,16 --new 192 \
      2>/dev/null | sed "s/^{/{\"push\": $push, /" >> $OUT || exit 1
  done
done
cat $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8 -o run -- \
  python3 tools/bench_decode.py --batches 1 --new 128 --tp-shard 8 > gpurun_out/r3m/p8.log 2>&1 || exit 1
python3 tools/trace_gaps.py /tmp/p8 > gpurun_out/r3m/p8_b1_gaps.txt 2>&1
head -10 gpurun_out/r3m/p8_b1_gaps.txt
