#!/bin/bash
# round 5: the RCCL ("nccl") process-group path of bench.py at world 1 (torchrun, MRSUM_FORCE_DIST=1): init,
# all-gather of summaries, barrier, timer all-reduce and the round-5 shutdown order -- exit code and JSON line
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MRSUM_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --hours 1 --steps 1 --warmup 1 \
  --max-new-tokens 64 > gpurun_out/r5_dist_world1_rccl.log 2>&1
rc=$?
echo "rc=$rc"
tail -n 1 gpurun_out/r5_dist_world1_rccl.log
exit $rc
