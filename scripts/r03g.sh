#!/bin/bash
# k_schur_tiles forms: C5 explicit timing per form + kernel stats, then the rig/explicit parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 1; do
  rm -rf gpurun_out/rigprof$f
  DAB_TILE_FORM=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rigprof$f -o run --output-format csv -- python3 scripts/rig_explicit.py 3 > gpurun_out/rigprof$f.log 2>&1
  rc=$?; grep -E "explicit|set_problem" gpurun_out/rigprof$f.log; [ $rc -eq 0 ] || exit $rc
  find gpurun_out/rigprof$f -name "*kernel_stats.csv" -exec cp {} gpurun_out/rig_stats$f.csv \;
  python3 - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/rig_stats{sys.argv[1]}.csv')))
for r in rows[:4]:
    print(f"form {sys.argv[1]}: {float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
done
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or explicit or tiles or c1" > gpurun_out/pytest_rig.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_rig.log
