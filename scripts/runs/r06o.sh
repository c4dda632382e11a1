#!/bin/bash
# round 6: the bulk update one work-group per super-tile (DAB_CHOL_BULK_GRID=0; the column
# updates beside it then get CUs as tiles finish) against the persistent grid of 448
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for g in 448 0 256; do
    echo "BULK_GRID=$g" >> $O/chol.txt
    DAB_CHOL_BULK_GRID=$g timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_CHOL_BULK_GRID=0 DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('BULK_GRID=0 vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
DAB_CHOL_BULK_GRID=0 DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
