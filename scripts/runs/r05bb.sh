#!/bin/bash
# camera-part split re-swept after the SGPR-constant series (the point waves' tables got cheaper):
# 800 / 840 (shipped) / 880 / 920 of 1024, C3, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05bb.txt; : > $O
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 5 s840 s800=LIB=scripts/ab/libdab_s800.so s880=LIB=scripts/ab/libdab_s880.so s920=LIB=scripts/ab/libdab_s920.so >> $O 2>&1 || { echo "ab rc=$?" >> $O; exit 1; }
