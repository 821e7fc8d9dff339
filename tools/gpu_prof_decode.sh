#!/bin/bash
# rocprofv3 kernel summaries of decode steps at fixed batch sizes (tools/bench_decode.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BATCHES:-1 39}; do
  NAME=profdec${TAG:-}_b$B
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/bench_decode.py --batches $B --new 128 ${EXTRA:-} > gpurun_out/$NAME.log 2>&1 || exit $?
  mkdir -p gpurun_out/$NAME
  python3 tools/trace_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  grep "^{" gpurun_out/$NAME.log
done
