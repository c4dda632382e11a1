#!/bin/bash
# Round-3 final binary: -m gpu suite, smoke, then traffic / bench / kernel stats (gpu_prof.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_u.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_u.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_u.log; [ $rc -eq 0 ] || exit $rc
TAG=r03u bash scripts/gpu_prof.sh
