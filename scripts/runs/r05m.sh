#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_SIDE=0 nopt=DAB_EVAL_SIDE=5 old=DAB_EVAL_BAL=0 > gpurun_out/r05m_abl_c3.log 2>&1
rc=$?; echo "abl rc=$rc"; tail -6 gpurun_out/r05m_abl_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_SIDE=0 old=DAB_EVAL_BAL=0 > gpurun_out/r05m_abl_c2.log 2>&1
rc=$?; echo "abl rc=$rc"; tail -4 gpurun_out/r05m_abl_c2.log; [ $rc -eq 0 ] || exit $rc
