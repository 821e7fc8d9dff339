#!/bin/bash
# Round 4: fused decode MLP of a TP shard -- kernel tests, tiny-model engine tests (they take the fused path
# at TP=1), then the TP=8 shard decode step with and without it (same box, interleaved).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4h
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "mlp_fused" --timeout 120 \
  --timeout-method thread > gpurun_out/r4h/test_mlp.log 2>&1 || { tail -30 gpurun_out/r4h/test_mlp.log; exit 1; }
tail -2 gpurun_out/r4h/test_mlp.log
true && \
true

for rep in 1 2; do
  for f in 0 1; do  # MRSUM_MLP_FUSED
    MRSUM_MLP_FUSED=$f timeout -k 10 200 python tools/bench_decode.py --tp-shard 8 --batches 1,5,10,16 --new 256 \
      > gpurun_out/r4h/shard8_fused$f.$rep.jsonl 2> gpurun_out/r4h/shard8_fused$f.$rep.err \
      || { tail -20 gpurun_out/r4h/shard8_fused$f.$rep.err; exit 1; }
    sed "s/^/fused=$f rep=$rep /" gpurun_out/r4h/shard8_fused$f.$rep.jsonl
  done
done
timeout -k 10 240 python tools/gemm_clock.py > gpurun_out/r4h/gemm_clock.jsonl 2> gpurun_out/r4h/gemm_clock.err \
  || { tail -20 gpurun_out/r4h/gemm_clock.err; exit 1; }
cat gpurun_out/r4h/gemm_clock.jsonl
