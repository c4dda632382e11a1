#!/bin/bash
# k_eval_bal camera waves' prologue records (bounds + first two steps' point indices built once
# per problem): fused-pass parity tests, then A/B against the round's record library (C3, C2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05ba.txt; : > $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_guard.py -k "fused or eval or split or guard or small" >> $O 2>&1 || { echo "pytest rc=$?" >> $O; exit 1; }
timeout -k 10 240 python -u scripts/eval_ab.py c3_1kcam 4 head=LIB=scripts/ab/libdab_head.so new >> $O 2>&1 || { echo "ab c3 rc=$?" >> $O; exit 1; }
timeout -k 10 240 python -u scripts/eval_ab.py c2_100cam 4 head=LIB=scripts/ab/libdab_head.so new >> $O 2>&1 || { echo "ab c2 rc=$?" >> $O; exit 1; }
