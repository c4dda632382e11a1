#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/trace6/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/r05h_trace6_c3.log 2>&1
echo "trace rc=$?"; head -12 gpurun_out/r05h_trace6_c3.log; tail -17 gpurun_out/r05h_trace6_c3.log
