#!/bin/bash
# round 3: full GPU suite + config-1 per-iteration timing (chol_prepare) + 2-rank AUTO rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u scripts/c1_iters.py > gpurun_out/c1_iters.log 2>&1
rc=$?; echo "c1 rc=$rc"; cat gpurun_out/c1_iters.log; [ $rc -eq 0 ] || exit $rc
