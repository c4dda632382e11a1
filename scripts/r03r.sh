#!/bin/bash
# k_schur_y at three waves per SIMD (half-wave record stage): C5 explicit kernel stats and
# the explicit / rig parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/syprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/syprof -o run --output-format csv -- python3 scripts/rig_explicit.py 4 > gpurun_out/syprof.log 2>&1 || { tail -5 gpurun_out/syprof.log; exit 1; }
grep -E "^explicit" gpurun_out/syprof.log
find gpurun_out/syprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/sy_stats.csv \;
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/sy_stats.csv')):
    if 'schur' in r['Name']:
        print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or explicit or tiles or c1 or setup" > gpurun_out/pytest_sy.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_sy.log
