#!/bin/bash
# round 6: k_eval_bal work-groups with no point slice skip the point tables (C2: the 99 camera work-groups), against the templated library
# (base = libdab_base13.so), 6 interleaved reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zl; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base13.so noslice"
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 6 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -3 $O/ab_c3.txt; grep "cost dev" $O/ab_c3.txt | awk '{print $NF}' | sort | uniq -c
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 6 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -3 $O/ab_c2.txt; grep "cost dev" $O/ab_c2.txt | awk '{print $NF}' | sort | uniq -c
