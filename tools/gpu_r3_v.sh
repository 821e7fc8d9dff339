#!/bin/bash
# Prefill attention: kernel tests of the final one-barrier variant, then PMC passes (own runs, kernel-trace only).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r3v
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context.py -k "prefill or long" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3v/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3v/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 python3 tools/pmc_attn.py > gpurun_out/r3v/plain.log 2>&1 || exit $?
i=0
for CTRS in "SQ_WAVE_CYCLES:SQ_WAIT_INST_LDS:SQ_WAIT_INST_ANY:SQ_WAIT_ANY:SQ_ACTIVE_INST_ANY:SQ_ACTIVE_INST_VALU:SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_WAVE_CYCLES:SQ_ACTIVE_INST_LDS:SQ_ACTIVE_INST_MISC:SQ_LDS_BANK_CONFLICT:SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $(echo $CTRS | tr : " ") --output-format csv -d /tmp/pa$i -o run -- \
    python3 tools/pmc_attn.py > gpurun_out/r3v/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r3v/pass$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pa$i > gpurun_out/r3v/pass$i.txt 2>&1
  cat gpurun_out/r3v/pass$i.txt
done
