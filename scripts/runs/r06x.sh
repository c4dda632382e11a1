#!/bin/bash
# round 6: k_eval_bal's point tables from the extrinsics' parameters staged by LDS-DMA
# (one request per line) instead of per-lane loads, C3 and C2, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06x; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="off=LIB=scripts/ab/libdab_extdma0.so on=LIB=scripts/ab/libdab_extdma1.so"
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 5 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -4 $O/ab_c3.txt
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 5 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -4 $O/ab_c2.txt
grep -h "cost dev" $O/ab_c3.txt | awk '{print $NF}' | sort | uniq -c
