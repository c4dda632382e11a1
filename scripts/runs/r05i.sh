#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 5 60 python -u scripts/xtab_probe.py c3_1kcam 1,0 > gpurun_out/r05i_probe_c3.log 2>&1
rc=$?; echo "probe c3 rc=$rc"; tail -3 gpurun_out/r05i_probe_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05i_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -3 gpurun_out/r05i_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05i_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -3 gpurun_out/r05i_ab_c2.log; [ $rc -eq 0 ] || exit $rc
DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/r05i_trace_c3.log 2>&1
echo "trace rc=$?"; head -12 gpurun_out/r05i_trace_c3.log; tail -17 gpurun_out/r05i_trace_c3.log
