#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_setup.py -q -m gpu --timeout 120 --timeout-method thread -x > gpurun_out/pytest_setup.log 2>&1
rc=$?; echo "setup tests rc=$rc"; tail -25 gpurun_out/pytest_setup.log; ok $rc || exit $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
DAB_SETUP_TIMING=1 timeout -k 10 300 python -u scripts/c5_check.py > gpurun_out/c5_setup.log 2>&1
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/c5_setup.log; ok $rc || exit $rc
timeout -k 10 120 python -u scripts/c1_iters.py
