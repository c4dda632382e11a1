#!/bin/bash
# the Cholesky column update (k_syrk_mfma) with unconditional clamped tile loads: Cholesky
# schedule parity tests, then n = 5994 factor + solve against the round's record library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05bd.txt; : > $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cholesky or dense or explicit" >> $O 2>&1 || { echo "pytest rc=$?" >> $O; exit 1; }
for r in 1 2 3; do
  for L in head new; do
    LIB=deeparc-sfm_amd/libdab.so; [ $L = head ] && LIB=scripts/ab/libdab_head.so
    echo "lib=$L" >> $O
    DAB_LIB=$LIB timeout -k 10 120 python -u scripts/chol_bench.py 5994 >> $O 2>&1 || exit 1
  done
done
