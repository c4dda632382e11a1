#!/bin/bash
# factor64 with the inverses off the chain: micro (accuracy vs CPU, phases), n = 5994 timing
# vs numpy, Cholesky / explicit-step tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 scripts/potrf_micro > gpurun_out/potrf_micro.log 2>&1
rc=$?; cat gpurun_out/potrf_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/chol_bench.py 5994 2>&1 | tail -2
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "chol or explicit or dense or c3 or c2 or spd" > gpurun_out/pytest_chol.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_chol.log
