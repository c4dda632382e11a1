#!/bin/bash
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) against the runtime default:
# one process per setting, interleaved, C3 and C2; then the prologue timeline with it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c3_1kcam c2_100cam; do
  for r in 1 2 3; do
    for k in unset 1 0; do
      if [ $k = unset ]; then
        timeout -k 10 120 env -u HIP_FORCE_DEV_KERNARG python -u scripts/eval_ab.py $c 1 bal > gpurun_out/r05y_${c}_${k}_$r.log 2>&1
      else
        HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python -u scripts/eval_ab.py $c 1 bal > gpurun_out/r05y_${c}_${k}_$r.log 2>&1
      fi
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/r05y_${c}_${k}_$r.log; exit $rc; }
      echo "$c kernarg=$k rep $r: $(tail -1 gpurun_out/r05y_${c}_${k}_$r.log)"
    done
  done
done
HIP_FORCE_DEV_KERNARG=1 DAB_TRACE_PER_WAVE=1 DAB_TRACE_PER_WG=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/r05y_trace_c3.log 2>&1
echo "trace rc=$?"; tail -1 gpurun_out/r05y_trace_c3.log
