#!/bin/bash
# round 6: the bulk update's grid (2 x CUs - F work-group slots left for the panel chain)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  for f in 64 32 96 128 160; do
    echo "BULK_FREE=$f" >> $O/chol.txt
    DAB_CHOL_BULK_FREE=$f timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  done
done
grep -v "^$" $O/chol.txt
