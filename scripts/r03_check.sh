#!/bin/bash
# Round-3 GPU check: parity tests, smoke, an A/B of the fused pass's camera-side forms at a
# new linearization point per pass (gather = default, stream = camera-major copy refreshed
# in the pass, fused = 16-B records), then the bench line. Stops at the first crash-type exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc


timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err; exit $rc
