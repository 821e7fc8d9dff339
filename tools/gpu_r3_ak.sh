#!/bin/bash
# Register-streaming (skinny) decode GEMMs with unconditional next-block prefetch: kernel / engine tests, then
# same-box decode-step A/B vs .ab_old (TP=1 and one rank's TP=8 shard, B=1/10 at 4k; 70B fp8 B=1 at 32k).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ak
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_forward_parity_gpu.py \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3ak/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3ak/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 1,10 --ctx 4000 --new 256 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3ak/ab.jsonl || exit 1
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 1,10 --ctx 4000 --new 256 --tp-shard 8 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3ak/ab.jsonl || exit 1
  done
done
for t in .ab_old .; do
  (cd $t && timeout -k 10 400 python tools/bench_decode.py --model llama3-70b --dtype fp8 --ctx 32000 --batches 1 --new 48 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3ak/ab.jsonl || exit 1
done
cat gpurun_out/r3ak/ab.jsonl
