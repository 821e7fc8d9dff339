#!/bin/bash
# round 5: is the 8-rank shared-GPU rehearsal's summary hash deterministic after the engine's window change, and
# what does the engine before that change give on the same box?  (1) current engine again; (2) the box's scratch
# copy of the package with engine.py from before the change (tools/_ab/engine_before_windows.py)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
run() {
  MRSUM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $1 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 \
    --max-new-tokens 32 --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r5_ii_$2.log 2>&1
  rc=$?
  grep "^{" gpurun_out/r5_ii_$2.log > gpurun_out/r5_ii_$2.json
  echo "$2 rc=$rc $(grep -o '"summary_sha16": "[0-9a-f]*"' gpurun_out/r5_ii_$2.json)"
  return $rc
}
run 29551 new || exit $?
cp tools/_ab/engine_before_windows.py llm_map_reduce_summarizer_amd/engine/engine.py
run 29552 old || exit $?
