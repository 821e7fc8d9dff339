#!/bin/bash
# round 5: the down projection on 8-wave workgroups x 8 splits (isolated: 22.0 vs 23.1 us at 39 rows,
# profiles/r2_stream_cfg_sweep_8b.jsonl) in situ at the headline's three decode phases
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
O=gpurun_out/r5_down_w8s8_insitu.jsonl
timeout -k 10 300 python -u tools/exp_plans_insitu.py --batch 39 --ctx 4400 --new 128 --variants plan,down:stream:8:8 >> $O 2>gpurun_out/r5_gg.err || exit $?
timeout -k 10 300 python -u tools/exp_plans_insitu.py --batch 10 --ctx 6000 --new 128 --variants plan,down:stream:8:8 >> $O 2>>gpurun_out/r5_gg.err || exit $?
timeout -k 10 300 python -u tools/exp_plans_insitu.py --batch 1 --ctx 13500 --new 128 --variants plan,down:stream:8:8 >> $O 2>>gpurun_out/r5_gg.err || exit $?
cat $O
