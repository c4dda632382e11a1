#!/bin/bash
# round 6: the fused column update at two waves per SIMD with its L_kk / inverse transfers in
# batches of 4 or 8 loads (32 / 48 B of scratch instead of 208), against the shipped instance
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for L in base6 chol_u4_lb chol_u8_lb; do
    echo "LIB=$L" >> $O/chol.txt
    DAB_LIB=scripts/ab/libdab_$L.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_LIB=scripts/ab/libdab_chol_u4_lb.so DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('u4_lb vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
DAB_LIB=scripts/ab/libdab_stamps_u4_lb.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
