#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 5 30 ./scripts/xcc_probe > gpurun_out/r05e_xcc.log 2>&1
rc=$?; echo "xcc rc=$rc"; cat gpurun_out/r05e_xcc.log
