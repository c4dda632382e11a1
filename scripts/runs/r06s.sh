#!/bin/bash
# round 6: y polling (r06r) with the y fill and the flag zeroing moved into the first panel launch
# then the values, against the round's previous library; bits; the dense and schedule tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for L in base6 new; do
    echo "LIB=$L" >> $O/chol.txt
    if [ $L = new ]; then X=; else X=scripts/ab/libdab_$L.so; fi
    DAB_LIB=$X timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print("y fill in the first panel vs r06c bitwise equal:", bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h "trsv" $O/prof/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_guard.py tests/test_gpu_reuse.py -k "dense or cholesky or explicit or guard or reuse" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
