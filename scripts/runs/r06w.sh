#!/bin/bash
# round 6: the column updates / strips with the next K chunk's loads issued before the
# current chunk's MFMAs, against the previous library; bits; stamps; C3 EXPLICIT; tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for L in base9 new; do
    echo "LIB=$L" >> $O/chol.txt
    if [ $L = new ]; then X=; else X=scripts/ab/libdab_$L.so; fi
    DAB_LIB=$X timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
    DAB_LIB=$X timeout -k 10 180 python3 scripts/explicit_run.py c3_1kcam >> $O/c3.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('chunk prefetch vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/c3.jsonl')]
for r in rows: print(r['lib'], round(r['iter_ms_median'],3))
print('costs identical:', len(set(tuple(r['costs']) for r in rows))==1)"
DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py -k "dense or cholesky" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
