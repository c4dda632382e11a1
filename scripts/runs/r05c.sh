#!/bin/bash
# k_eval_bal (per-XCD tables built once in the launch, shared camera frames) against
# k_eval_fused: A/B at C3 and C2, then the -m gpu suite on k_eval_bal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05c_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -4 gpurun_out/r05c_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05c_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -4 gpurun_out/r05c_ab_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05c_pytest.log; exit $rc
