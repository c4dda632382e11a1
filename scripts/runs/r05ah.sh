#!/bin/bash
# C2: waves per camera capped at 4 / 2 (DAB_FUSED_WPC; the default takes 8 at C2); one
# process per setting (the cap is read once)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for w in 0 4 2; do
    DAB_FUSED_WPC=$w timeout -k 10 120 python -u scripts/eval_ab.py c2_100cam 1 bal > gpurun_out/r05ah_$w_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
    echo "wpc cap $w rep $r: $(tail -1 gpurun_out/r05ah_$w_$r.log)"
  done
done
