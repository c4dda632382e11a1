#!/bin/bash
# round 6: per-work-group phase stamps of one n = 5994 factorisation (a -DDAB_CHOL_STAMPS
# build): where the chain's column updates and the bulk spend their time beside each other
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
grep -c stamps $O/stamps.txt; tail -2 $O/stamps.txt
