#!/bin/bash
# config 1's set-up and first solve under a kernel trace: device time per kernel against the
# wall-clock phases (scripts/c1_first.py, DAB_SETUP_TIMING=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
rm -rf gpurun_out/r05ap_trace
DAB_SETUP_TIMING=1 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r05ap_trace -o run --output-format csv -- python3 scripts/c1_first.py > gpurun_out/r05ap.log 2>&1
echo "rc=$?"; grep "^rep" gpurun_out/r05ap.log
