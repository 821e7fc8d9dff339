#!/bin/bash
# Decode step decomposition: the per-launch fixed cost + streaming rate of a graph-captured dependent kernel
# chain (tools/exp_launch_floor.py), and rocprofv3 kernel traces of the decode steps it is meant to explain:
# Llama-3-70B fp8 B=1 at 32k (config 5) and Llama-3-8B bf16 B=1 at 13.5k (the headline's final reduce).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r4w
export TMPDIR=/tmp
timeout -k 10 180 python tools/exp_launch_floor.py > gpurun_out/r4w/launch_floor.jsonl 2> gpurun_out/r4w/launch_floor.err \
  || { tail -5 gpurun_out/r4w/launch_floor.err; exit 1; }
cat gpurun_out/r4w/launch_floor.jsonl
BATCHES=1 TAG=_70b32k EXTRA="--model llama3-70b --dtype fp8 --ctx 32000" bash tools/gpu_prof_decode.sh || exit 1
BATCHES=1 TAG=_8b13k EXTRA="--ctx 13500" bash tools/gpu_prof_decode.sh || exit 1
