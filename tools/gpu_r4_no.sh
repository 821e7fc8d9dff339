#!/bin/bash
# Round 4: in-situ decode attention plans at the level-1 (B = 5 / 16, class <= 12k) and final-reduce (B = 1,
# ~13.5k, class <= 32k) shapes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
bash tools/gpu_r4_n.sh && bash tools/gpu_r4_o.sh
