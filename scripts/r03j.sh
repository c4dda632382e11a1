#!/bin/bash
# device tile tables: device-vs-host set-up bitwise tests, rig/explicit parity, first-solve
# timing (C3, C5) and config-1 per-iteration timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "setup or rig or c5 or explicit or tiles or c1 or host" > gpurun_out/pytest_rig.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_rig.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DAB_SETUP_TIMING=1 timeout -k 10 300 python3 -u scripts/first_solve.py > gpurun_out/first_solve.log 2>&1
rc=$?; grep -E "solve|set_problem |schur_t|build_schur" gpurun_out/first_solve.log | head -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/c1_iters.py > gpurun_out/c1_iters.log 2>&1
rc=$?; cat gpurun_out/c1_iters.log; [ $rc -eq 0 ] || exit $rc
