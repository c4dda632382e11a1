#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_SIDE=0 empty=DAB_EVAL_SIDE=4 nopt=DAB_EVAL_SIDE=5 nofr=DAB_EVAL_SIDE=6 > gpurun_out/r05l_abl_c3.log 2>&1
rc=$?; echo "abl rc=$rc"; tail -7 gpurun_out/r05l_abl_c3.log; [ $rc -eq 0 ] || exit $rc
