#!/bin/bash
# dense Cholesky with the bulk's first block column as its own launch (DAB_CHOL_STRIP=1)
# against the default: n = 5994 timing (interleaved), dense tests, timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for r in 1 2; do
  for st in 0 1; do
    DAB_CHOL_STRIP=$st timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/r05ai_$st_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/r05ai_$st_$r.log; exit $rc; }
    echo "strip=$st rep $r: $(tail -1 gpurun_out/r05ai_$st_$r.log)"
  done
done
DAB_CHOL_STRIP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r05ai_dense.log 2>&1
echo "dense tests rc=$?"; tail -1 gpurun_out/r05ai_dense.log
rm -rf gpurun_out/r05ai_trace
DAB_CHOL_STRIP=1 timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r05ai_trace -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > gpurun_out/r05ai_trace.log 2>&1
echo "trace rc=$?"
python3 scripts/chol_timeline.py gpurun_out/r05ai_trace > gpurun_out/r05ai_timeline.txt 2>&1; sed -n 1,30p gpurun_out/r05ai_timeline.txt
