#!/bin/bash
# k_eval_bal after the claim-loop fix: correctness probe (C2, C3), A/B against k_eval_fused,
# per-wave timelines (trace build scripts/trace5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in c2_100cam c3_1kcam; do
  timeout -k 5 60 python -u scripts/xtab_probe.py $c 1,0 > gpurun_out/r05f_probe_$c.log 2>&1
  rc=$?; echo "probe $c rc=$rc"; tail -4 gpurun_out/r05f_probe_$c.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u scripts/eval_ab.py c3_1kcam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05f_ab_c3.log 2>&1
rc=$?; echo "ab c3 rc=$rc"; tail -3 gpurun_out/r05f_ab_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/eval_ab.py c2_100cam 3 bal=DAB_EVAL_BAL=1 fused=DAB_EVAL_BAL=0 > gpurun_out/r05f_ab_c2.log 2>&1
rc=$?; echo "ab c2 rc=$rc"; tail -3 gpurun_out/r05f_ab_c2.log; [ $rc -eq 0 ] || exit $rc
for c in c3_1kcam c2_100cam; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/trace5/libdab.so timeout -k 5 90 python -u scripts/trace_fused.py $c > gpurun_out/r05f_trace_$c.log 2>&1
  echo "trace $c rc=$?"
done
