#!/bin/bash
# End-of-session rehearsal of bench.py's N>1 paths on the 1-GPU box: world 1 with RCCL forced on, 2 ranks
# sharing the GPU (gloo) as the planner chooses, and 8 ranks sharing it with map TP=2 x DP=4 + TP=8 final.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4z
MRSUM_FORCE_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 1 --hours 1 --steps 1 --warmup 1 \
  --max-new-tokens 64 > gpurun_out/r4z/world1_rccl.log 2>&1 || { tail -20 gpurun_out/r4z/world1_rccl.log; exit 1; }
grep "^{" gpurun_out/r4z/world1_rccl.log | cut -c1-400
( export MRSUM_DP_KV_FRACTION=0.15 MRSUM_REDUCE_KV_FRACTION=0.15 ENGINE_KV_FRACTION=0.15
  MRSUM_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29582 bench.py --gpus 2 --hours 1 --steps 1 --warmup 1 --max-new-tokens 64 \
    --parallel auto > gpurun_out/r4z/gloo2_auto.log 2>&1 ) || { tail -20 gpurun_out/r4z/gloo2_auto.log; exit 1; }
grep "^{" gpurun_out/r4z/gloo2_auto.log | cut -c1-400
( export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
  MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29583 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
    --parallel map:tp2,reduce_final:tp8 > gpurun_out/r4z/gloo8_tp.log 2>&1 ) \
  || { tail -20 gpurun_out/r4z/gloo8_tp.log; exit 1; }
grep "^{" gpurun_out/r4z/gloo8_tp.log | cut -c1-400
grep -o '"timed_work": {[^}]*}' gpurun_out/r4z/*.log
