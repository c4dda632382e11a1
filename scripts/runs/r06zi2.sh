#!/bin/bash
# round 6 (second sweep, 8 reps): k_eval_bal camera split (first part of a two-part chunk, in 1/1024) re-swept on
# the final kernel (the frames' affine chunk map moved the camera prologue), C3, 4 reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zi2; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="s840 s900=DAB_CAM_SPLIT=900 s1000=DAB_CAM_SPLIT=1000 s1016=DAB_CAM_SPLIT=1016"
timeout -k 10 500 python -u scripts/eval_ab.py c3_1kcam 8 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -8 $O/ab_c3.txt
