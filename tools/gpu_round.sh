#!/bin/bash
# One GPU session: kernel/engine tests, smoke, short + headline bench.
# A test FAILURE (pytest rc 1) does not stop the session; a crash, abort or
# timeout (any other non-zero rc) ends it immediately (no further GPU work).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
[ "${BENCH:-1}" = "1" ] || exit 0
step bench_1h 600 python bench.py --hours 1 --steps 1 --warmup 1 --log-level INFO || exit $?
step bench_10h 900 python bench.py --steps 2 --warmup 1 --log-level INFO || exit $?
