#!/bin/bash
# Round 4 multi-process rehearsal on one GPU: (1) torchrun world 1 over RCCL (the N > 1 code path of bench.py,
# incl. the pinned-work check), (2) 8 ranks sharing the GPU over gloo with the planner's auto layout and
# (3) map TP=2 x DP=4 + a TP=8 final reduce (8-peer custom all-reduce, TP push, per-generate error vote).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4f
MRSUM_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --hours 1 --steps 1 --warmup 1 \
  --max-new-tokens 64 > gpurun_out/r4f/world1_rccl.log 2>&1 || { tail -5 gpurun_out/r4f/world1_rccl.log; exit 1; }
grep "^{" gpurun_out/r4f/world1_rccl.log | cut -c1-400
export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
  --log-level INFO > gpurun_out/r4f/rehearsal_8rank_auto.log 2>&1 || { tail -20 gpurun_out/r4f/rehearsal_8rank_auto.log; exit 1; }
grep "^{" gpurun_out/r4f/rehearsal_8rank_auto.log | cut -c1-600
MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
  --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r4f/rehearsal_8rank_tp8.log 2>&1 || { tail -20 gpurun_out/r4f/rehearsal_8rank_tp8.log; exit 1; }
grep "^{" gpurun_out/r4f/rehearsal_8rank_tp8.log | cut -c1-600
