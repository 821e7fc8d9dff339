#!/bin/bash
# Iteration session: targeted GPU tests, then the microbenchmarks named in $STEPS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-it}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py ${TESTK:+-k "$TESTK"} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
for st in ${STEPS:-}; do
  case $st in
    tpshard) timeout -k 10 300 python tools/bench_tp_shard.py > gpurun_out/${T}_tpshard.log 2>&1 || exit $? ;;
    dec8) timeout -k 10 300 python tools/bench_decode.py --tp-shard 8 --batches 1,10,39 > gpurun_out/${T}_dec8.log 2>&1 || exit $? ;;
    dec4) timeout -k 10 300 python tools/bench_decode.py --tp-shard 4 --batches 1,10,39 > gpurun_out/${T}_dec4.log 2>&1 || exit $? ;;
    dec1) timeout -k 10 300 python tools/bench_decode.py --batches 1,10,39 > gpurun_out/${T}_dec1.log 2>&1 || exit $? ;;
    bench) timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $? ;;
  esac
  echo "step $st done"
done
