#!/bin/bash
# PMC counter sets over one command (each set its own rocprofv3 run under its own time
# limit; a set that fails is reported and skipped, a timed-out one ends the script).
# Usage: TAG=name FILTER=k_eval bash scripts/pmc_sets.sh "SET1" "SET2" ... -- cmd args
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
TAG=${TAG:-pmc}; OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
sets=()
while [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- "$@" > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then echo "pass $i ($set) timed out"; exit $rc; fi
  [ $rc -eq 0 ] || { echo "pass $i ($set) failed rc=$rc"; tail -3 $OUT/p$i.log; }
done
FILTER="${FILTER:-k_}" OUT=$OUT python3 - <<'PY'
import csv, glob, collections, os
flt, out = os.environ["FILTER"], os.environ["OUT"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dab::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    if flt not in k: continue
    print(k, "launches", len(next(iter(agg[k].values()))))
    for c, v in sorted(agg[k].items()):
        print(f"   {c:34s} {sum(v)/len(v):18.1f}")
PY
