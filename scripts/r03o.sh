#!/bin/bash
# rig pair-kernel point pre-gather A/B (DAB_PAIR_GATHER 1 | 0): LM times of the rig mixed
# PCG run and the kernel stats of the pair kernel and the gather
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 1 0; do
  rm -rf gpurun_out/pgprof$g
  DAB_PAIR_GATHER=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pgprof$g -o run --output-format csv -- python3 scripts/rig_mixed.py 3 > gpurun_out/pgprof$g.log 2>&1 || exit 1
  echo "== DAB_PAIR_GATHER=$g"; grep -E "^mixed|^fp64" gpurun_out/pgprof$g.log | head -4
  find gpurun_out/pgprof$g -name "*kernel_stats.csv" -exec cp {} gpurun_out/pg_stats$g.csv \;
  python3 - $g <<'PY'
import csv, sys
for r in csv.DictReader(open(f'gpurun_out/pg_stats{sys.argv[1]}.csv')):
    if 'pair' in r['Name']:
        print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
done
DAB_PAIR_GATHER=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or pair or reuse or setup" > gpurun_out/pytest_pg.log 2>&1
rc=$?; echo "pytest (gather on) rc=$rc"; tail -4 gpurun_out/pytest_pg.log
