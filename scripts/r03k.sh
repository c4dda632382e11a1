#!/bin/bash
# rig mixed PCG: the product's camera-sum forms (DAB_MF32_ACC 0/1/2) -> per-iteration time,
# CG counts against the oracle, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in ${FORMS:-0 1 2}; do
  rm -rf gpurun_out/mixprof$f
  DAB_MF32_ACC=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mixprof$f -o run --output-format csv -- python3 scripts/rig_mixed.py 5 > gpurun_out/mixprof$f.log 2>&1
  rc=$?; echo "== acc form $f"; grep -v "^W2026\|simple_timer" gpurun_out/mixprof$f.log | tail -8; [ $rc -eq 0 ] || exit $rc
  find gpurun_out/mixprof$f -name "*kernel_stats.csv" -exec cp {} gpurun_out/mix_stats$f.csv \;
  python3 - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/mix_stats{sys.argv[1]}.csv')))
for r in rows[:10]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
done
