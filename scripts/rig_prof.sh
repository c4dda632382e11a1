#!/bin/bash
# GPU box: kernel stats of the config-5 check (scripts/c5_check.py) and its LM summary lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/rigtr
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rigtr -o run --output-format csv -- python3 scripts/c5_check.py "$@" > gpurun_out/rigtr.log 2>&1 || { tail -5 gpurun_out/rigtr.log; exit 1; }
grep -E "iter|obs/s|eval" gpurun_out/rigtr.log | tail -6
find gpurun_out/rigtr -name "*kernel_stats.csv" -exec cp {} gpurun_out/rig_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/rig_stats.csv')))
for r in rows[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
PY
