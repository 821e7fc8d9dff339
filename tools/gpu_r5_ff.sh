#!/bin/bash
# round 5: LDS-DMA stream with no compute vs the stream GEMM vs the register-load probe (tools/exp_stream_dma.py)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/exp_stream_dma.py > gpurun_out/r5_stream_dma.jsonl 2> gpurun_out/r5_stream_dma.err
rc=$?; echo "rc=$rc"; tail -n 3 gpurun_out/r5_stream_dma.err; exit $rc
