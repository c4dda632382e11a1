#!/bin/bash
# the camera-part split of k_eval_bal (kCamSplit, in 1/1024; tuned at 688 for round 3's
# kernel) re-swept: one process per value (read once), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2 3 4; do
  for sp in 688 840 900 960; do
    DAB_CAM_SPLIT=$sp timeout -k 10 120 python -u scripts/eval_ab.py c3_1kcam 1 bal > gpurun_out/r05aq_${sp}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/r05aq_${sp}_$r.log; exit $rc; }
    echo "split $sp rep $r: $(tail -1 gpurun_out/r05aq_${sp}_$r.log)"
  done
done
