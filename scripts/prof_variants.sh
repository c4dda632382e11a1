#!/bin/bash
# GPU box: eval_variants.py under rocprofv3 kernel trace; prints per-kernel average ns
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
CFG=$1; shift
rm -rf gpurun_out/pv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv -o run --output-format csv -- python3 scripts/eval_variants.py $CFG "$@" > gpurun_out/pv.log 2>&1 || { tail -20 gpurun_out/pv.log; exit 1; }
grep "$CFG" gpurun_out/pv.log
find gpurun_out/pv -name "*kernel_stats.csv" -exec cp {} gpurun_out/pv_stats.csv \;
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/pv_stats.csv')):
    if 'eval' in r['Name'] or 'KERNEL_FILTER' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.2f} us  min {float(r['MinNs'])/1e3:8.2f}  n={r['Calls']:>4}  {r['Name'][:90]}")
PY
