#!/bin/bash
# 8 ranks sharing the GPU over gloo: the world-8 paths the driver's N=8 scaling run takes (auto layout
# from the planner; then map TP=2 x DP=4 with the final reduce on a TP=8 engine, i.e. an 8-peer custom
# all-reduce and the TP push in the o / down epilogues).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ar
# eight ranks share one card: a small KV pool each (0.03 ran the card out of memory with two engines a rank)
export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
if [ "${SKIP_AUTO:-0}" != 1 ]; then
MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
  --log-level INFO > gpurun_out/r3ar/rehearsal_8rank_auto.log 2>&1 || exit 1
grep "^{" gpurun_out/r3ar/rehearsal_8rank_auto.log | cut -c1-700
fi
MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
  --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r3ar/rehearsal_8rank_tp8.log 2>&1 || exit 1
grep "^{" gpurun_out/r3ar/rehearsal_8rank_tp8.log | cut -c1-700
