set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/base
timeout -k 10 300 python3 tools/bench_decode.py --batches 1,10,39 --new 256 > gpurun_out/base/tp1.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_decode.py --batches 1,10,39 --new 256 --tp-shard 8 > gpurun_out/base/tp8.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p8 -o run -- python3 tools/bench_decode.py --batches 1 --new 128 --tp-shard 8 > gpurun_out/base/p8.log 2>&1 || exit $?
python3 tools/trace_summary.py /tmp/p8 > gpurun_out/base/p8_summary.txt 2>&1
python3 tools/trace_gaps.py /tmp/p8 > gpurun_out/base/p8_gaps.txt 2>&1
grep -h "^{" gpurun_out/base/*.log
