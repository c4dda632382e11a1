#!/bin/bash
# strips on a third stream (DAB_CHOL_STRIP3=1: the bulk starts as soon as its panel is done)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for st in 0 1; do
    DAB_CHOL_STRIP3=$st timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/r05ak_${st}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/r05ak_${st}_$r.log; exit $rc; }
    echo "strip3=$st rep $r: $(tail -1 gpurun_out/r05ak_${st}_$r.log | cut -c1-90)"
  done
done
DAB_CHOL_STRIP3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05ak_dense.log 2>&1
echo "dense tests rc=$?"; tail -1 gpurun_out/r05ak_dense.log
