#!/bin/bash
# PMC counters of the kernels whose names match $FILTER while running "$@" (each counter set
# its own rocprofv3 run, every run under its own time limit). Prints the per-launch means.
# Usage: FILTER=k_mf_frame bash scripts/pmc_kernels.sh python3 scripts/rig_mixed.py 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmck && export TMPDIR=/tmp
rm -rf gpurun_out/pmck/p*
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d gpurun_out/pmck/p$i -o run --output-format csv -- "$@" > gpurun_out/pmck/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmck/p$i.log; exit 1; }
done
FILTER="${FILTER:-k_}" python3 - <<'PY'
import csv, glob, collections, os
flt = os.environ["FILTER"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmck/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dab::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    if flt not in k: continue
    print(k, "launches", len(next(iter(agg[k].values()))))
    for c, v in sorted(agg[k].items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}")
PY
