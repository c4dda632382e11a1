#!/bin/bash
# camera-wave prologue reorder: per-wave traces (C2, C3), quick bench (headline + C2), -m gpu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DAB_TRACE_LIB=scripts/trace2/libdab.so timeout -k 10 120 python -u scripts/trace_fused.py c2_100cam > gpurun_out/trace2_c2.log 2>&1 || exit $?
DAB_TRACE_PER_WAVE=1 DAB_TRACE_LIB=scripts/trace2/libdab.so timeout -k 10 120 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/trace2_c3.log 2>&1 || exit $?
head -12 gpurun_out/trace2_c2.log; head -1 gpurun_out/trace2_c3.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-lm --no-rig --no-c4 --no-c1 > gpurun_out/bench_q$i.json 2> gpurun_out/bench_q$i.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_q$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d.get('c2_eval_ms_per_step',0)*1e3, d.get('c2_eval_kernel_ms',0)*1e3)"
done
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_s.log; exit $rc
