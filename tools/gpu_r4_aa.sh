#!/bin/bash
# A/B/A/B on one box: decode attention partials stored plain (default) vs write-through (MRSUM_ATTN_PART_WT=1)
# for the separate split merge; whole decode steps at the headline's three phase shapes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4aa
for r in 1 2; do
  for wt in 0 1; do
    for cfg in "1 13500" "10 6000" "39 4400"; do
      set -- $cfg
      MRSUM_ATTN_PART_WT=$wt timeout -k 10 200 python tools/bench_decode.py --batches $1 --ctx $2 --new 256 \
        2> gpurun_out/r4aa/err.log | sed "s|^{|{\"part_wt\": $wt, \"round\": $r, |" | tee -a gpurun_out/r4aa/ab.jsonl || exit 1
    done
  done
done
