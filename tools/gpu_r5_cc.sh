set -e
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5_cc_engine_tests.txt 2>&1
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_bench_windows.json 2> gpurun_out/r5_bench_windows.err
