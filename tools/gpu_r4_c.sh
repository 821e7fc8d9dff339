#!/bin/bash
# Round 4: fp8 KV cache -- kernel + engine + parity tests, decode-step A/B (bf16 vs fp8 KV) at the map / reduce
# batch sizes, and the labelled fp8-KV variant of the headline bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4c
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_forward_parity_gpu.py \
  -k "attn or rope or fp8_kv or gqa or eos or parity or two_term or rmsnorm_fp8 or gemm_fp8" -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r4c/tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "parity|passed|failed|Error|error" gpurun_out/r4c/tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for kv in bf16 fp8; do
  timeout -k 10 300 python tools/bench_decode.py --batches 1,10,39 --ctx 4400 --new 128 --kv-dtype $kv \
    >> gpurun_out/r4c/decode_ab.jsonl 2> gpurun_out/r4c/decode_$kv.err || { tail -5 gpurun_out/r4c/decode_$kv.err; exit 1; }
done
cat gpurun_out/r4c/decode_ab.jsonl
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --kv-dtype fp8 > gpurun_out/r4c/bench_fp8kv.json 2> gpurun_out/r4c/bench_fp8kv.err
rc=$?; echo "bench fp8kv rc=$rc"; tail -3 gpurun_out/r4c/bench_fp8kv.err
python -c "import json; d=json.load(open('gpurun_out/r4c/bench_fp8kv.json')); print('bench fp8kv', d['ms_per_step'], d['value'], d['timed_work'], d['phases_s'], d['reduce_plan']['seconds'])"
exit $rc
