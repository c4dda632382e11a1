#!/bin/bash
# camera waves building half of the point tables (DAB_EVAL_SIDE=32) at C3 / C2, the C2 grid
# A/B, then the -m gpu suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_SIDE=0 ctab=DAB_EVAL_SIDE=32 > gpurun_out/r05w_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -3 gpurun_out/r05w_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_SIDE=0 ctab=DAB_EVAL_SIDE=32 > gpurun_out/r05w_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -3 gpurun_out/r05w_ab_c2.log; [ $rc -eq 0 ] || exit $rc
DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/r05w_trace_c3.log 2>&1
echo "trace rc=$?"; tail -14 gpurun_out/r05w_trace_c3.log
bash scripts/runs/r05v.sh
