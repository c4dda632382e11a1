#!/bin/bash
# C2 grid A/B (r05u), then the -m gpu suite on the current library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/runs/r05u.sh || exit $?
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05v_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r05v_pytest_gpu.log; exit $rc
