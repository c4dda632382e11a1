#!/bin/bash
# the half-tile bulk update (C prefetch) on top of the column-update load fix: Cholesky parity
# tests, then n = 5994 against the column-fix library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05be.txt; : > $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cholesky or dense or explicit" >> $O 2>&1 || { echo "pytest rc=$?" >> $O; exit 1; }
for r in 1 2 3; do
  for L in col new; do
    LIB=deeparc-sfm_amd/libdab.so; [ $L = col ] && LIB=scripts/ab/libdab_col.so
    echo "lib=$L" >> $O
    DAB_LIB=$LIB timeout -k 10 120 python -u scripts/chol_bench.py 5994 >> $O 2>&1 || exit 1
  done
done
