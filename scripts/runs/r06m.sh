#!/bin/bash
# round 6: the bulk stream on a CU mask (DAB_CHOL_CUMASK=R reserves R CUs for the chain), so
# that the chain's column updates (one work-group per CU) find whole free CUs beside the bulk
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
run() { echo "$1" >> $O/chol.txt; env $1 timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1; }
for rep in 1 2; do
  run "DAB_CHOL_CUMASK=0" || exit 1
  run "DAB_CHOL_CUMASK=32" || exit 1
  run "DAB_CHOL_CUMASK=64" || exit 1
  run "DAB_CHOL_CUMASK=32 DAB_CHOL_NOGRAPH=1" || exit 1
  run "DAB_CHOL_CUMASK=0 DAB_CHOL_NOGRAPH=1" || exit 1
done
DAB_CHOL_CUMASK=32 DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x.npy'); print('CUMASK=32 vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
grep -v "^$" $O/chol.txt
DAB_CHOL_CUMASK=32 DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps32.txt 2>&1 || { tail $O/stamps32.txt; exit 1; }
