#!/bin/bash
# the frame builder issuing the intrinsic with the extrinsic: new vs previous library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c2_100cam c3_1kcam; do
  timeout -k 10 300 python -u scripts/eval_ab.py $c 4 prev=LIB=scripts/trace6/libdab_prev.so new=LIB=scripts/trace6/libdab_new.so > gpurun_out/r05ab_$c.log 2>&1
  rc=$?; echo "ab $c rc=$rc"; tail -3 gpurun_out/r05ab_$c.log; [ $rc -eq 0 ] || exit $rc
done
