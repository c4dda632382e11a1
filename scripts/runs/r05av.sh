#!/bin/bash
# Cholesky: the strip on a third stream beside the bulk (DAB_CHOL_STRIP=2, new default) against
# the strip in front of the bulk (1) and the base library
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05av.txt; : > $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "cholesky or dense" >> $O 2>&1 || { echo "pytest rc=$?" >> $O; exit 1; }
for r in 1 2 3; do
  for V in base:1 cur:1 cur:2 halves:2 halves:1; do
    L=${V%%:*}; S=${V##*:}
    LIB=deeparc-sfm_amd/libdab.so; [ $L = base ] && LIB=scripts/ab/libdab_base.so; [ $L = halves ] && LIB=scripts/ab/libdab_halves.so
    echo "lib=$L strip=$S" >> $O
    DAB_CHOL_STRIP=$S DAB_LIB=$LIB timeout -k 10 120 python -u scripts/chol_bench.py 5994 >> $O 2>&1 || exit 1
  done
done
