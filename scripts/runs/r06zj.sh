#!/bin/bash
# round 6: k_eval_bal with a role split (DAB_EVAL_ROLES=kp: work-groups 0..kp-1 run the point
# side with all 16 waves, the others the camera side with all 16) against the fused
# schedule (8 + 8 waves in every work-group; base = the shipped library), C3 and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zj; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base12.so fused r104=DAB_EVAL_ROLES=104 r112=DAB_EVAL_ROLES=112 r120=DAB_EVAL_ROLES=120 r128=DAB_EVAL_ROLES=128 r128e=DAB_EVAL_ROLES=128,DAB_CAM_SPLIT=512 r112e=DAB_EVAL_ROLES=112,DAB_CAM_SPLIT=512"
timeout -k 10 500 python -u scripts/eval_ab.py c3_1kcam 3 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -9 $O/ab_c3.txt; grep "cost dev" $O/ab_c3.txt | awk '{print $NF}' | sort | uniq -c
V="base=LIB=scripts/ab/libdab_base12.so fused r64=DAB_EVAL_ROLES=64 r128=DAB_EVAL_ROLES=128 r192=DAB_EVAL_ROLES=192"
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -6 $O/ab_c2.txt; grep "cost dev" $O/ab_c2.txt | awk '{print $NF}' | sort | uniq -c
