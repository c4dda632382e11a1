#!/bin/bash
# round 6: k_eval_bal's camera pipeline depth (points gathered DG steps ahead, indices DI,
# R register slots): 2/4/3 (shipped) against 2/5/3, 3/6/4, 3/7/4 at C3 and C2, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V=""; for v in 243 253 364 374; do V="$V cam$v=LIB=scripts/ab/libdab_cam$v.so"; done
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 4 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -8 $O/ab_c3.txt
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 4 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -8 $O/ab_c2.txt
