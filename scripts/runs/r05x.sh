#!/bin/bash
# per-wave timeline with the prologue hops (trace build), C3 and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c3_1kcam c2_100cam; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py $c > gpurun_out/r05x3_trace_$c.log 2>&1
  echo "trace $c rc=$?"; tail -3 gpurun_out/r05x3_trace_$c.log
done
