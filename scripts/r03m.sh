#!/bin/bash
# handle-reuse tests, then the round-3 profile set (traffic PMC, bench line, kernel trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_reuse.py -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_reuse.log 2>&1
rc=$?; echo "reuse pytest rc=$rc"; tail -15 gpurun_out/pytest_reuse.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=${TAG:-r03b} bash scripts/gpu_prof.sh > gpurun_out/prof_${TAG:-r03b}.log 2>&1
rc=$?; tail -45 gpurun_out/prof_${TAG:-r03b}.log; exit $rc
