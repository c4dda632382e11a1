#!/bin/bash
# camera-chunk split share A/B at C3 (trace builds; kernel mean over 50 passes + per-wave timeline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in trace_base trace_x640 trace_x688 trace_x600; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/$v/libdab.so timeout -k 10 120 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/t_${v}_$rep.log 2>&1 || exit $?
  echo "$v rep $rep: $(head -1 gpurun_out/t_${v}_$rep.log)"
done
done
