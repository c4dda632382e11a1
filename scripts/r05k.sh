#!/bin/bash
# k_eval_bal table-phase ablations at C3 (timing only) and the TAB form (tables of the current x
# from a k_cam_tables launch in front, as the LM loop's candidate provides them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 both=DAB_EVAL_SIDE=0 tables=DAB_EVAL_SIDE=3 tabcopy=DAB_EVAL_SIDE=3,DAB_FUSED_TAB=1 empty=DAB_EVAL_SIDE=4 tab=DAB_FUSED_TAB=1 oldtab=DAB_EVAL_BAL=0,DAB_FUSED_TAB=1 > gpurun_out/r05k_abl_c3.log 2>&1
rc=$?; echo "abl rc=$rc"; tail -7 gpurun_out/r05k_abl_c3.log
