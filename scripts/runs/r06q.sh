#!/bin/bash
# round 6: the (lean) strip on a third stream beside the bulk (DAB_CHOL_STRIP=3) against the
# strip launch in front of the bulk on the bulk stream (=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for m in 1 3; do
    echo "STRIP=$m" >> $O/chol.txt
    DAB_CHOL_STRIP=$m timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_CHOL_STRIP=3 DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('STRIP=3 vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
DAB_CHOL_STRIP=3 DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "cholesky" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
