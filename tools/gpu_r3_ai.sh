#!/bin/bash
# Headline bench with larger packed prefill passes (MRSUM_MAX_PREFILL_TOKENS) and prefill slices
# (MRSUM_PREFILL_CHUNK), alternating with the defaults, 2 timed steps each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3ai
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/r3ai/$tag.json 2> gpurun_out/r3ai/$tag.err \
    || { tail -3 gpurun_out/r3ai/$tag.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r3ai/$tag.json')); e=d['engine_rank0']; print('$tag', d['ms_per_step'], e['prefill_s'], e['prefill_tok_s'], e['decode_s'])"
}
run base MRSUM_X=0 || exit 1
run p32k MRSUM_MAX_PREFILL_TOKENS=32768 || exit 1
run p64k MRSUM_MAX_PREFILL_TOKENS=65536 || exit 1
run p32k_c8k MRSUM_MAX_PREFILL_TOKENS=32768 MRSUM_PREFILL_CHUNK=8192 || exit 1
run base2 MRSUM_X=0 || exit 1
