#!/bin/bash
# k_schur_tiles (matrix-core form): rig explicit parity tests, then C5 timing + kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or explicit or tiles or c1" > gpurun_out/pytest_rig.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_rig.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/rig_explicit.py 4 > gpurun_out/rig_explicit.log 2>&1
rc=$?; cat gpurun_out/rig_explicit.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/rigprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rigprof -o run --output-format csv -- python3 scripts/rig_explicit.py 3 > gpurun_out/rigprof.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
find gpurun_out/rigprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/rig_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/rig_stats.csv')))
for r in rows[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
PY
