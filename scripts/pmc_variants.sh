#!/bin/bash
# GPU box: PMC counters of the evaluation kernels for eval_variants.py variants (one
# rocprofv3 pass per counter set, each under its own time limit). Prints per-kernel means.
# usage: scripts/pmc_variants.sh CONFIG VARIANT [VARIANT ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcv && export TMPDIR=/tmp
CFG=$1; shift
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  rm -rf gpurun_out/pmcv/p$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmcv/p$i -o run --output-format csv -- python3 scripts/eval_variants.py $CFG "$@" > gpurun_out/pmcv/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcv/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmcv/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dab::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    if not k.startswith("k_eval"): continue
    print(k)
    for c, v in sorted(agg[k].items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}")
PY
