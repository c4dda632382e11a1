#!/bin/bash
# GPU box check: parity tests, smoke, short bench. Stops at the first crash-type exit
# (fault/abort/segv/timeout); plain test failures (rc 1) do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; exit $rc
