#!/bin/bash
# rocprofv3 kernel-trace + stats of a short end-to-end bench (10 h transcript, 128 new tokens per call).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NAME=${NAME:-prof}
timeout -k 10 ${TO:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$NAME -o run -- \
  python3 bench.py --steps 1 --warmup 1 --max-new-tokens ${NEW:-128} ${EXTRA} > gpurun_out/$NAME.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 3 gpurun_out/$NAME.log; exit $rc
