#!/bin/bash
# (1) the reference-compatible CLI end to end on the local engine (1 h synthetic transcript, report +
#     intermediate chunk summaries); (2) the 70B fp8 aggregator on a TP=2 engine whose two ranks share
#     the GPU (gloo for host collectives, IPC P2P all-reduce fused with RMSNorm at hidden 8192, fp8
#     decode GEMMs at TP shard shapes, vocab-parallel sampling).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cli
python3 -c "
import json, sys
sys.path.insert(0, '.')
from llm_map_reduce_summarizer_amd.utils.synth import synthetic_transcript
json.dump(synthetic_transcript(1.0, seed=5, n_speakers=2), open('gpurun_out/cli/talk.json', 'w'))" || exit 1
timeout -k 10 400 python3 -m llm_map_reduce_summarizer_amd -i gpurun_out/cli/talk.json -o gpurun_out/cli/summary.md \
  --report --save-chunks gpurun_out/cli/chunks.json --max-new-tokens 64 > gpurun_out/cli/cli.log 2>&1 || exit $?
python3 -c "
import json; r = json.load(open('gpurun_out/cli/summary.report.json'))
print('cli report:', {k: r[k] for k in ('chunks', 'segments', 'tokens_used', 'provider', 'model', 'processing_time')})" || exit 1
MRSUM_DIST_BACKEND=gloo ENGINE_KV_FRACTION=0.2 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/bench_aggregator.py --context 8000 \
  --max-new-tokens 64 > gpurun_out/agg_tp2.log 2>&1 || exit $?
grep '"value"' gpurun_out/agg_tp2.log
