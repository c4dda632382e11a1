#!/bin/bash
# round 6: panels per bulk update (DAB_CHOL_GROUP 2 / 3 / 4) on the round-6 kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  for g in 2 3 4; do
    echo "GROUP=$g" >> $O/chol.txt
    DAB_CHOL_GROUP=$g timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
grep -v "^$" $O/chol.txt
