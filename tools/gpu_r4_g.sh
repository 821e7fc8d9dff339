#!/bin/bash
# Round 4: 8-rank shared-GPU rehearsal of map TP=2 x DP=4 + TP=8 final reduce (CP fallback path), then the 24 h
# transcript (2-level reduce) and the 24 h single-pass Llama-3.1 reduce, bf16 KV and fp8 KV.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4g
( export MRSUM_DP_KV_FRACTION=0.01 MRSUM_REDUCE_KV_FRACTION=0.01 ENGINE_KV_FRACTION=0.01
  MRSUM_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 8 --hours 1 --steps 1 --warmup 0 --max-new-tokens 32 \
    --parallel map:tp2,reduce_final:tp8 --log-level INFO > gpurun_out/r4g/rehearsal_8rank_tp8.log 2>&1 ) \
  || { tail -20 gpurun_out/r4g/rehearsal_8rank_tp8.log; exit 1; }
grep "^{" gpurun_out/r4g/rehearsal_8rank_tp8.log | cut -c1-300
grep -o '"timed_work": {[^}]*}' gpurun_out/r4g/rehearsal_8rank_tp8.log
for kv in bf16 fp8; do
  timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 --kv-dtype $kv > gpurun_out/r4g/bench24h_$kv.json \
    2> gpurun_out/r4g/bench24h_$kv.err || { tail -5 gpurun_out/r4g/bench24h_$kv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4g/bench24h_$kv.json')); print('24h $kv', d['ms_per_step'], d['value'], d['timed_work'], d['reduce_plan']['calls'])"
  timeout -k 10 400 python bench.py --hours 24 --steps 1 --warmup 1 --model llama3.1-8b --no-hierarchical --kv-dtype $kv \
    > gpurun_out/r4g/bench24h_single_$kv.json 2> gpurun_out/r4g/bench24h_single_$kv.err || { tail -5 gpurun_out/r4g/bench24h_single_$kv.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r4g/bench24h_single_$kv.json')); print('24h single-pass $kv', d['ms_per_step'], d['value'], d['timed_work'], d['phases_s'])"
done
