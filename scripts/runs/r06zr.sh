#!/bin/bash
# round 6: per-wave timeline of the final k_eval_bal (trace build, prologue hops), C2 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zr; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c2_100cam c3_1kcam; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/ab/trace/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py $c > $O/trace_$c.log 2>&1
  echo "trace $c rc=$?"; tail -3 $O/trace_$c.log
done
