#!/bin/bash
# (1) B=39 / B=10 in-situ: deferred norm up to 64 rows, attention split counts;
# (2) Llama-3-70B fp8 TP=8 shard decode step at 32k, B=1;
# (3) 4 ranks sharing the GPU over gloo with per-stage TP x DP layouts (map TP=2 x DP=2, final TP=4).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3h
OUT=gpurun_out/r3h/plans.jsonl
: > $OUT
run() { timeout -k 10 400 python tools/exp_plans_insitu.py "$@" 2>/dev/null >> $OUT || exit 1; }
run --batch 39 --variants plan,defer64,attnsep4,attnsep6,attnsep2
run --batch 10 --variants plan,defer8
cat $OUT
timeout -k 10 400 python tools/bench_decode.py --model llama3-70b --dtype fp8 --tp-shard 8 --batches 1,10 --ctx 32000 \
  --new 128 > gpurun_out/r3h/tp8_70b_fp8.log 2>&1 || exit 1
grep "^{" gpurun_out/r3h/tp8_70b_fp8.log
timeout -k 10 500 python tools/bench_decode.py --model llama3-70b --dtype fp8 --batches 1 --ctx 32000 \
  --new 128 > gpurun_out/r3h/tp1_70b_fp8.log 2>&1 || exit 1
grep "^{" gpurun_out/r3h/tp1_70b_fp8.log
export MRSUM_DP_KV_FRACTION=0.05 MRSUM_REDUCE_KV_FRACTION=0.05 ENGINE_KV_FRACTION=0.05
MRSUM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --hours 1 --steps 1 --warmup 1 --max-new-tokens 64 \
  --parallel map:tp2,reduce_final:tp4 --log-level INFO > gpurun_out/r3h/rehearsal_4rank_layouts.log 2>&1 || exit 1
grep "^{" gpurun_out/r3h/rehearsal_4rank_layouts.log | cut -c1-600
