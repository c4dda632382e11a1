#!/bin/bash
# Round-4 record: -m gpu suite, smoke, then traffic / bench / kernel stats (gpu_prof.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_z.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_z.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_z.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -2 gpurun_out/smoke_z.log; [ $rc2 -eq 0 ] || exit $rc2
TAG=r04z bash scripts/gpu_prof.sh
exit $rc
