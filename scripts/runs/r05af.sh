#!/bin/bash
# dense Cholesky at n = 5994 (C3's reduced camera system): timing and per-step timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/r05af_chol.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/r05af_chol.log
rm -rf gpurun_out/r05af_trace
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r05af_trace -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > gpurun_out/r05af_trace.log 2>&1
echo "trace rc=$?"
python3 scripts/chol_timeline.py gpurun_out/r05af_trace > gpurun_out/r05af_timeline.txt 2>&1
echo "timeline rc=$?"; head -12 gpurun_out/r05af_timeline.txt
