#!/bin/bash
# Rehearse the multi-process paths on a 1-GPU box:
#  (1) torchrun world=1 with the RCCL ("nccl") backend forced on: process group, RCCL all-gather of
#      summaries, device barrier, all_reduce(max) of the timer -- the N>1 code path of bench.py;
#  (2) two ranks sharing cuda:0 over gloo, every stage data-parallel: DP scatter / all-gather with two
#      GPU engines;
#  (3) the same two ranks with the reduce stages tensor-parallel (TP=2 engine: custom P2P all-reduce
#      inside the decode hipGraphs, vocab-parallel sampling, gloo for the eager prefill all-reduces);
#  (4) every stage on the TP=2 engine (--parallel tp) and (5) the planner's choice (--parallel auto;
#      its measured all-reduce constants are those of two ranks sharing one GPU, not of xGMI).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
MRSUM_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --hours 1 --steps 1 --warmup 1 \
  --max-new-tokens 64 > gpurun_out/dist_world1_rccl.log 2>&1 || exit $?
tail -n 1 gpurun_out/dist_world1_rccl.log
export MRSUM_DP_KV_FRACTION=0.15 MRSUM_REDUCE_KV_FRACTION=0.15 ENGINE_KV_FRACTION=0.15
MRSUM_DIST_BACKEND=gloo MRSUM_PARALLEL=dp timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --hours 1 --steps 1 \
  --warmup 1 --max-new-tokens 64 > gpurun_out/dist_gloo2_shared_gpu.log 2>&1 || exit $?
tail -n 1 gpurun_out/dist_gloo2_shared_gpu.log
MRSUM_DIST_BACKEND=gloo MRSUM_PARALLEL=reduce_tp timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --hours 1 --steps 1 \
  --warmup 1 --max-new-tokens 64 --log-level INFO > gpurun_out/dist_gloo2_reduce_tp.log 2>&1 || exit $?
tail -n 1 gpurun_out/dist_gloo2_reduce_tp.log
port=29520
for mode in tp auto; do
port=$((port + 1))  # a fresh rendezvous port per run (the previous one may linger in TIME_WAIT)
MRSUM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --hours 1 --steps 1 \
  --warmup 1 --max-new-tokens 64 --parallel $mode --log-level INFO > gpurun_out/dist_gloo2_$mode.log 2>&1 || exit $?
tail -n 1 gpurun_out/dist_gloo2_$mode.log
done
