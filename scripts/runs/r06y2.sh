#!/bin/bash
# round 6: is the C5 PCG product bound by its sweep-2 fp64 LDS atomics in both precisions?
# (1) kernel times of k_mf_frame<0> (fp64) and k_mf_frame32 (mixed) with the atomics and in a
# -DDAB_ABL_MF_NOSUMS build (sums into a register: timing only); (2) PART=pmc: their LDS and
# issue counters on the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06y2; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ "${PART:-time}" = time ]; then
  for L in prod nosums; do
    for f in 0 1; do
      if [ $L = prod ]; then X=; else X=scripts/ab/libdab_mfnosums.so; fi
      rm -rf $O/t_${L}_$f
      DAB_LIB=$X timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t_${L}_$f -o run --output-format csv -- python3 scripts/rig_pcg_run.py c5_rig_16x64 $f > $O/t_${L}_$f.log 2>&1 || { echo "run $L $f failed"; tail -3 $O/t_${L}_$f.log; exit 1; }
      echo "$L fp32=$f: $(grep -h iter_ms_median $O/t_${L}_$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["iter_ms_median"],3), d["cg"])')"
      grep -h -E "k_mf_frame<0>|k_mf_frame32|k_mf_diag_frame" $O/t_${L}_$f/run_kernel_stats.csv | cut -d, -f1-4
    done
  done
  exit 0
fi
for f in 0 1; do
  FILTER=k_mf_frame bash scripts/pmc_kernels.sh python3 scripts/rig_pcg_run.py c5_rig_16x64 $f > $O/pmc_$f.txt 2>&1 || { echo "pmc $f failed"; tail -5 $O/pmc_$f.txt; exit 1; }
  cat $O/pmc_$f.txt
done
