#!/bin/bash
# k_schur_tiles half-block form (C5 kernel stats) + device pair tables (first-solve timing,
# device-vs-host set-up bitwise tests, rig/explicit parity tests)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/r03h.sh || exit $?
DAB_SETUP_TIMING=1 timeout -k 10 300 python3 -u scripts/first_solve.py > gpurun_out/first_solve.log 2>&1
rc=$?; grep -E "solve|set_problem|pairs|schur_t|build_schur" gpurun_out/first_solve.log | head -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_setup.py tests/test_gpu_full_size.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_setup.log 2>&1
rc=$?; echo "setup/full-size pytest rc=$rc"; tail -5 gpurun_out/pytest_setup.log
