#!/bin/bash
# k_eval_bal phase ablations at C3 and C2 (timing only; wrong results by design)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c3_1kcam c2_100cam; do
timeout -k 10 200 python -u scripts/eval_ab.py $c 3 both=DAB_EVAL_SIDE=0 point=DAB_EVAL_SIDE=1 camera=DAB_EVAL_SIDE=2 tables=DAB_EVAL_SIDE=3 old=DAB_EVAL_BAL=0 > gpurun_out/r05j_abl_$c.log 2>&1
rc=$?; echo "abl $c rc=$rc"; tail -6 gpurun_out/r05j_abl_$c.log; [ $rc -eq 0 ] || exit $rc
done
