#!/bin/bash
# Decode attention with a true two-tile prefetch (steady loop without per-tile branches): attention tests, then
# same-box A/B vs .ab_old: standalone kernel (B=1 at 10k / 32k, B=10 / 39 at 4.4k), whole decode steps
# (TP=1 B=1 at 10k, B=10 / 39 at 4k, TP=8 shard B=1) and the 70B fp8 B=1 32k decode.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3aq
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py tests/test_engine_gpu.py tests/test_forward_parity_gpu.py \
  -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3aq/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3aq/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_attn_decode.py --batches 1 --ctx 10000 --rounds 2 | sed "s|^{|{\"tree\": \"$t\", |") | grep "^{" >> gpurun_out/r3aq/kern.jsonl || exit 1
    (cd $t && timeout -k 10 300 python tools/bench_attn_decode.py --batches 1 --ctx 32000 --rounds 2 | sed "s|^{|{\"tree\": \"$t\", |") | grep "^{" >> gpurun_out/r3aq/kern.jsonl || exit 1
    (cd $t && timeout -k 10 300 python tools/bench_attn_decode.py --batches 10,39 --ctx 4400 --rounds 2 | sed "s|^{|{\"tree\": \"$t\", |") | grep "^{" >> gpurun_out/r3aq/kern.jsonl || exit 1
  done
done
cat gpurun_out/r3aq/kern.jsonl
for r in 1 2; do
  for t in .ab_old .; do
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 1 --ctx 10000 --new 256 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3aq/steps.jsonl || exit 1
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 10,39 --ctx 4000 --new 256 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3aq/steps.jsonl || exit 1
    (cd $t && timeout -k 10 300 python tools/bench_decode.py --batches 1 --ctx 4000 --new 256 --tp-shard 8 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3aq/steps.jsonl || exit 1
  done
done
for t in .ab_old .; do
  (cd $t && timeout -k 10 400 python tools/bench_decode.py --model llama3-70b --dtype fp8 --ctx 32000 --batches 1 --new 48 | sed "s|^{|{\"tree\": \"$t\", |") >> gpurun_out/r3aq/steps.jsonl || exit 1
done
cat gpurun_out/r3aq/steps.jsonl
