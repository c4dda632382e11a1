#!/bin/bash
# C2: the single fused launch at smaller grids (DAB_FUSED_GRID)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 g256=DAB_FUSED_GRID=0 g192=DAB_FUSED_GRID=192 g128=DAB_FUSED_GRID=128 g100=DAB_FUSED_GRID=100 g64=DAB_FUSED_GRID=64 > gpurun_out/r05u_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -6 gpurun_out/r05u_ab_c2.log; [ $rc -eq 0 ] || exit $rc
