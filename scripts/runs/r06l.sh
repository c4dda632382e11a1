#!/bin/bash
# round 6: the group's first column update (beside the bulk) without the fused panel step
# (DAB_CHOL_F_SPLIT=1: its work-groups do not wait for the diagonal factor; the panel rows are
# solved by k_panel after it); lean strips (k_syrk_mfma<false>)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for f in 0 1; do
    echo "F_SPLIT=$f" >> $O/chol.txt
    DAB_CHOL_F_SPLIT=$f timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
for f in 0 1; do
  DAB_CHOL_F_SPLIT=$f DAB_DUMP=$O/x$f.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x$f.npy'); print('F_SPLIT=$f vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
done
grep -v "^$" $O/chol.txt
DAB_CHOL_F_SPLIT=1 DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps2.txt 2>&1 || { tail $O/stamps2.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py -k "dense or cholesky" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; exit $rc
