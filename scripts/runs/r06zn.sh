#!/bin/bash
# round 6: C2 with fewer waves per camera (DAB_EVAL_WPC=4 / 2: two / four cameras per
# work-group, 4 / 8 steps per wave) against the shipped 8 (one camera per work-group)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zn; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base14.so w8 w4=DAB_EVAL_WPC=4 w2=DAB_EVAL_WPC=2"
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 6 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -5 $O/ab_c2.txt; grep "cost dev" $O/ab_c2.txt | awk '{print $NF}' | sort | uniq -c
