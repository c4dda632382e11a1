#!/bin/bash
# k_syrk_big with unconditional clamped loads (new) against the previous build: n = 5994,
# interleaved; the dense tests on the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in prev new; do
    DAB_LIB=scripts/trace6/libdab_$v.so timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/r05am_${v}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/r05am_${v}_$r.log; exit $rc; }
    echo "$v rep $r: $(tail -1 gpurun_out/r05am_${v}_$r.log | cut -c1-90)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05am_dense.log 2>&1
echo "dense tests rc=$?"; tail -1 gpurun_out/r05am_dense.log
