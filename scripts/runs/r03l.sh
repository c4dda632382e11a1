#!/bin/bash
# dense Cholesky n = 5994: timing and a kernel-trace timeline of the last factorisation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/chol_bench.py 5994 ${CHOL_ENV:+} 2>&1 | tail -2
rm -rf gpurun_out/cholprof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/cholprof -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > gpurun_out/cholprof.log 2>&1 || { tail -5 gpurun_out/cholprof.log; exit 1; }
python3 scripts/chol_timeline.py gpurun_out/cholprof 400 > gpurun_out/chol_timeline.txt
head -12 gpurun_out/chol_timeline.txt
