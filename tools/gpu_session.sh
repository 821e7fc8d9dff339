mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s5_pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/s5_pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/s5_bench10h.json 2> gpurun_out/s5_bench10h.err || exit $?
cat gpurun_out/s5_bench10h.json
timeout -k 10 300 python tools/bench_decode.py --tp-shard 8 --batches 1,5,10,39 > gpurun_out/s5_tp8shard.log 2>&1 || exit $?
cat gpurun_out/s5_tp8shard.log
