#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python -u scripts/xtab_probe.py c2_100cam > gpurun_out/r05d_c2.log 2>&1
rc=$?; echo "c2 rc=$rc"; tail -12 gpurun_out/r05d_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xtab_probe.py c3_1kcam > gpurun_out/r05d_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -12 gpurun_out/r05d_c3.log; exit $rc
