#!/bin/bash
# round 6: the back substitution by owner pairs (DAB_CHOL_BACK_PAIRS=1) against single-block
# owners (=0): n = 5994 interleaved, bits, kernel time, C3 EXPLICIT, the dense tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06y3}; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for m in 0 1; do
    echo "BACK_PAIRS=$m" >> $O/chol.txt
    DAB_CHOL_BACK_PAIRS=$m timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('owner pairs vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
for m in 0 1; do
  DAB_CHOL_BACK_PAIRS=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$m -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > $O/prof$m.log 2>&1 || { echo "prof failed"; exit 1; }
  grep -h "trsv" $O/prof$m/run_kernel_stats.csv | cut -d, -f1-4
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "dense or cholesky or explicit" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
