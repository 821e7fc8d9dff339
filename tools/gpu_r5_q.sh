#!/bin/bash
# round 5: the 8-rank shared-GPU rehearsal of round 4 (profiles/r4_rehearsal_8rank_tp8_cp_fallback.json: map TP=2 x DP=4,
# final reduce on a TP=8 engine whose o / down GEMMs push over an 8-peer custom all-reduce, 1 % KV pools so the
# context-parallel prefill falls back) on this round's kernels -- pinned work and the summary hash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
MRSUM_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 \
  --max-new-tokens 32 --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r5_rehearsal_8rank.log 2>&1
rc=$?
grep "^{" gpurun_out/r5_rehearsal_8rank.log > gpurun_out/r5_rehearsal_8rank.json
echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
# the same with round 4's 4-wave register-streaming kernels (their fp32 summation order)
MRSUM_SKINNY_WAVES=4 MRSUM_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 \
  --max-new-tokens 32 --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r5_rehearsal_8rank_w4.log 2>&1
rc=$?
grep "^{" gpurun_out/r5_rehearsal_8rank_w4.log > gpurun_out/r5_rehearsal_8rank_w4.json
echo "rc=$rc"
exit $rc
