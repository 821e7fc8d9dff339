#!/bin/bash
# rocprofv3 kernel traces of the headline's other two decode phases at their real shapes: level-1 reduce
# (B=10 at ~6k context) and map (B=39 at ~4.4k).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
BATCHES=10 TAG=_8b6k EXTRA="--ctx 6000" bash tools/gpu_prof_decode.sh || exit 1
BATCHES=39 TAG=_8b4k4 EXTRA="--ctx 4400" bash tools/gpu_prof_decode.sh || exit 1
