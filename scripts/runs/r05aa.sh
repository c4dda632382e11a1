#!/bin/bash
# point waves holding their K LDS-DMA (32) / all their table loads (64) until the camera waves
# have issued their first gathers; timelines of both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_SIDE=0 holdK=DAB_EVAL_SIDE=32 holdAll=DAB_EVAL_SIDE=64 > gpurun_out/r05aa_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -4 gpurun_out/r05aa_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_SIDE=0 holdK=DAB_EVAL_SIDE=32 holdAll=DAB_EVAL_SIDE=64 > gpurun_out/r05aa_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -4 gpurun_out/r05aa_ab_c2.log; [ $rc -eq 0 ] || exit $rc
for sd in 32 64; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py c3_1kcam $sd > gpurun_out/r05aa_trace_c3_$sd.log 2>&1
  echo "trace $sd rc=$?"; tail -1 gpurun_out/r05aa_trace_c3_$sd.log
done
