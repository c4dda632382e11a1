#!/bin/bash
# the strip schedule (now the default) with the bulk grid leaving 64 (default), 32, 0 or 96
# work-group slots (two per CU) to the chain: n = 5994, interleaved, one process each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for f in 64 32 0 96 128; do
    DAB_CHOL_BULK_FREE=$f timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/r05aj_${f}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/r05aj_${f}_$r.log; exit $rc; }
    echo "free=$f rep $r: $(tail -1 gpurun_out/r05aj_${f}_$r.log | cut -c1-80)"
  done
done
