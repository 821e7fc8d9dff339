#!/bin/bash
# rocprofv3 kernel-trace of a short end-to-end bench (10 h transcript, NEW tokens per call): the stats
# CSVs, a per-kernel summary and the decode-step busy / gap accounting come back under gpurun_out/NAME/.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
NAME=${NAME:-prof}
OUT=/tmp/$NAME
timeout -k 10 ${TO:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 1 --warmup 1 --max-new-tokens ${NEW:-1000} ${EXTRA:-} > gpurun_out/$NAME.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 3 gpurun_out/$NAME.log
mkdir -p gpurun_out/$NAME
find $OUT -name "*stats.csv" -exec cp {} gpurun_out/$NAME/ \;
python3 tools/trace_summary.py $OUT > gpurun_out/$NAME/summary.txt 2>&1 || true
exit $rc
