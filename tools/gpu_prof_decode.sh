#!/bin/bash
# rocprofv3 kernel traces of decode steps at fixed batch sizes (tools/bench_decode.py): per-kernel
# summary + per-step kernel-busy / gap accounting (tools/trace_gaps.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BATCHES:-1 39}; do
  NAME=profdec${TAG:-}_b$B
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/$NAME -o run -- \
    python3 tools/bench_decode.py --batches $B --new 128 ${EXTRA:-} > gpurun_out/$NAME.log 2>&1 || exit $?
  mkdir -p gpurun_out/$NAME
  python3 tools/trace_summary.py /tmp/$NAME > gpurun_out/$NAME/summary.txt 2>&1
  python3 tools/trace_gaps.py /tmp/$NAME > gpurun_out/$NAME/gaps.txt 2>&1
  grep "^{" gpurun_out/$NAME.log
  head -40 gpurun_out/$NAME/gaps.txt
done
