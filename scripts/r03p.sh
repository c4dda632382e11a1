#!/bin/bash
# round-3 final: the whole -m gpu suite, then the profile set (traffic PMC of this binary,
# bench line, kernel trace) under TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_final.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=${TAG:-r03c} bash scripts/gpu_prof.sh > gpurun_out/prof_${TAG:-r03c}.log 2>&1
rc=$?; tail -8 gpurun_out/prof_${TAG:-r03c}.log | cut -c1-600; exit $rc
