#!/bin/bash
# the camera waves' first loads before the work-group's first barrier (DAB_EVAL_SIDE 32: the
# chunk bounds and frame records, 64: also the first indices); timelines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_SIDE=0 early1=DAB_EVAL_SIDE=32 early2=DAB_EVAL_SIDE=64 > gpurun_out/r05ad_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -4 gpurun_out/r05ad_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_SIDE=0 early1=DAB_EVAL_SIDE=32 early2=DAB_EVAL_SIDE=64 > gpurun_out/r05ad_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -4 gpurun_out/r05ad_ab_c2.log; [ $rc -eq 0 ] || exit $rc
for sd in 32 64; do
  for c in c3_1kcam c2_100cam; do
    DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py $c $sd > gpurun_out/r05ad_trace_${c}_$sd.log 2>&1
    echo "trace $c $sd rc=$?"; tail -1 gpurun_out/r05ad_trace_${c}_$sd.log
  done
done
