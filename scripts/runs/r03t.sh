#!/bin/bash
# camera-chunk split share A/B at C3 (trace builds; kernel mean over 50 passes + per-wave timeline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in trace_base trace_stage2; do
  DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/$v/libdab.so timeout -k 10 120 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/t_${v}_$rep.log 2>&1 || exit $?
  echo "$v rep $rep: $(head -1 gpurun_out/t_${v}_$rep.log)"
done
done
if [ -n "$WITH_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu --no-lm --no-rig --no-c4 --no-c1 > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_t.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d.get('c2_eval_kernel_ms',0)*1e3)"
fi
