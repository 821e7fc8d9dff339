#!/bin/bash
# round 5: the fused (in-launch, last-arriver) split merge at 32 splits for one decode row -- the kernel sweep
# had it 0.7 us faster at 13.5k (r5_attn_decode_b1_splits_pmc.txt) -- in situ against the separate merge
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5_v_fused32_insitu.jsonl
timeout -k 10 300 python tools/exp_plans_insitu.py --batch 1 --ctx 13500 --variants plan,attnfused32,attnfused24 >> $OUT 2>/dev/null || exit $?
timeout -k 10 600 python tools/exp_plans_insitu.py --model llama3-70b --dtype fp8 --batch 1 --ctx 32000 --new 96 --variants plan,attnfused32,resid:o=skinny,resid:down=skinny >> $OUT 2>/dev/null || exit $?
cat $OUT
