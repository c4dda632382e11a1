#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 3 base=DAB_EVAL_SIDE=0 map688=DAB_EVAL_SIDE=32 map600=DAB_EVAL_SIDE=39321632 map560=DAB_EVAL_SIDE=36700192 map640=DAB_EVAL_SIDE=41943072 map740=DAB_EVAL_SIDE=48496672 > gpurun_out/r05p_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -7 gpurun_out/r05p_ab_c3.log; [ $rc -eq 0 ] || exit $rc
