#!/bin/bash
# round 5, after the engine's pinned-window / one-sync-admission change: tools/gpu_r5_q.sh's 8-rank shared-GPU
# rehearsal (map TP=2 x DP=4, TP=8 final reduce over the 8-peer P2P all-reduce, CP fallback) -- pinned work,
# every P2P path self-tested, and the summary hash of the same build (a4fcbfbb45caecc0) unchanged
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
MRSUM_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 \
  --max-new-tokens 32 --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r5_rehearsal_8rank_final.log 2>&1
rc=$?
grep "^{" gpurun_out/r5_rehearsal_8rank_final.log > gpurun_out/r5_rehearsal_8rank_final.json
echo "rc=$rc"
exit $rc
