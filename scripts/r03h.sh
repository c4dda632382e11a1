#!/bin/bash
# k_schur_tiles timing (C5 explicit, kernel stats) then the rig/explicit parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/rigprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rigprof -o run --output-format csv -- python3 scripts/rig_explicit.py ${ITERS:-3} > gpurun_out/rigprof.log 2>&1
rc=$?; grep -E "explicit|set_problem" gpurun_out/rigprof.log; [ $rc -eq 0 ] || exit $rc
find gpurun_out/rigprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/rig_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/rig_stats.csv')))
for r in rows[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "${TESTK:-rig or c5 or explicit or tiles or c1}" > gpurun_out/pytest_rig.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_rig.log
