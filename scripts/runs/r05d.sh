#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 5 30 ./scripts/xtab_harness > gpurun_out/r05d_harness.log 2>&1; echo "harness rc=$?"; cat gpurun_out/r05d_harness.log
for m in 0 4 3 2; do
  timeout -k 5 25 python -u scripts/xtab_probe.py c2_100cam $m > gpurun_out/r05d_c2_m$m.log 2>&1
  echo "mode $m rc=$?"; tail -6 gpurun_out/r05d_c2_m$m.log
done
