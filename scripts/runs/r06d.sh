#!/bin/bash
# round 6: the strip's tiles inside the chain's column update (DAB_CHOL_STRIP=2) against the
# strip launch on the bulk stream (=1): n = 5994 factor + solve interleaved, bits against r06c,
# the timeline of =2, the schedule-agreement and dense tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for m in 1 2; do
    echo "STRIP=$m" >> $O/chol.txt
    DAB_CHOL_STRIP=$m timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
DAB_CHOL_STRIP=2 DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('strip on the chain vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
cat $O/chol.txt
DAB_CHOL_STRIP=2 timeout -k 10 180 rocprofv3 --kernel-trace -d $O/chol_trace -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > $O/chol_trace.log 2>&1 || { echo "chol trace failed"; tail $O/chol_trace.log; exit 1; }
python3 scripts/chol_timeline.py $O/chol_trace 80 > $O/chol_timeline.txt 2>&1; sed -n 1,12p $O/chol_timeline.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py \
  -k "dense or cholesky" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; exit $rc
