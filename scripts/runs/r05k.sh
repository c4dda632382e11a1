#!/bin/bash
# series Rodrigues tables: k_eval_bal phase ablations at C3 (timing only), the TAB form, the old
# kernel; then the -m gpu suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 both=DAB_EVAL_SIDE=0 tables=DAB_EVAL_SIDE=3 tabcopy=DAB_EVAL_SIDE=3,DAB_FUSED_TAB=1 empty=DAB_EVAL_SIDE=4 tab=DAB_FUSED_TAB=1 old=DAB_EVAL_BAL=0 > gpurun_out/r05k_abl_c3.log 2>&1
rc=$?; echo "abl rc=$rc"; tail -7 gpurun_out/r05k_abl_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_BAL=1 old=DAB_EVAL_BAL=0 tables=DAB_EVAL_SIDE=3 > gpurun_out/r05k_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -4 gpurun_out/r05k_ab_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05k_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05k_pytest.log; exit $rc
