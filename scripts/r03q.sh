#!/bin/bash
# k_schur_tiles load balance (DAB_TILE_BALANCE 1 | 0): C5 explicit LM timing + kernel stats,
# then the explicit / rig parity tests with the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1 0; do
  rm -rf gpurun_out/tbprof$b
  DAB_TILE_BALANCE=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tbprof$b -o run --output-format csv -- python3 scripts/rig_explicit.py 4 > gpurun_out/tbprof$b.log 2>&1 || { tail -5 gpurun_out/tbprof$b.log; exit 1; }
  echo "== DAB_TILE_BALANCE=$b"; grep -E "^explicit" gpurun_out/tbprof$b.log
  find gpurun_out/tbprof$b -name "*kernel_stats.csv" -exec cp {} gpurun_out/tb_stats$b.csv \;
  python3 - $b <<'PY'
import csv, sys
for r in csv.DictReader(open(f'gpurun_out/tb_stats{sys.argv[1]}.csv')):
    if 'schur' in r['Name']:
        print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
done
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or explicit or tiles or c1 or setup or reuse or dist" > gpurun_out/pytest_tb.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_tb.log
