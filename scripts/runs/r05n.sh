#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_SIDE=0 old=DAB_EVAL_BAL=0 > gpurun_out/r05n_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -3 gpurun_out/r05n_ab_c2.log; [ $rc -eq 0 ] || exit $rc
for c in c3_1kcam c2_100cam; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py $c > gpurun_out/r05n_trace_$c.log 2>&1
  echo "trace $c rc=$?"
done
