#!/bin/bash
# the -m gpu suite under DAB_DEV_POISON=1 on the round's final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_DEV_POISON=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05ay_pytest_poison.log 2>&1
rc=$?; echo "poison rc=$rc"; tail -3 gpurun_out/r05ay_pytest_poison.log; exit $rc
