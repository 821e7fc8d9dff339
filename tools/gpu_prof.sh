#!/bin/bash
# rocprofv3 kernel-trace + stats of a short end-to-end bench (10 h transcript, NEW tokens per call).
# Full traces stay on the box (/tmp); only the stats CSVs + a per-kernel summary come back.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
NAME=${NAME:-prof}
OUT=/tmp/$NAME
timeout -k 10 ${TO:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 1 --warmup 1 --max-new-tokens ${NEW:-128} ${EXTRA} > gpurun_out/$NAME.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 3 gpurun_out/$NAME.log
mkdir -p gpurun_out/$NAME
find $OUT -name "*stats.csv" -exec cp {} gpurun_out/$NAME/ \;
python3 tools/trace_summary.py $OUT > gpurun_out/$NAME/summary.txt 2>&1 || true
exit $rc
