#!/bin/bash
# round 6: k_eval_bal's camera split (first part of a two-part chunk, in 1/1024) re-swept on
# the final kernel (the frames' affine chunk map moved the camera prologue), C3, 4 reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zi; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="s840 s720=DAB_CAM_SPLIT=720 s780=DAB_CAM_SPLIT=780 s900=DAB_CAM_SPLIT=900 s960=DAB_CAM_SPLIT=960 s1000=DAB_CAM_SPLIT=1000"
timeout -k 10 500 python -u scripts/eval_ab.py c3_1kcam 4 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -8 $O/ab_c3.txt
