#!/bin/bash
# rig preconditioner pass k_mf_diag_frame at 3 waves per SIMD (launch bounds, 53 VGPRs spilled)
# against 2 (224 VGPRs): C5 PCG LM iteration, fp64 and mixed, interleaved; kernel stats of each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05az.txt; : > $O
for r in 1 2; do
  for L in cur mf3; do
    for F in 0 1; do
      echo "lib=$L fp32=$F" >> $O
      DAB_LIB=scripts/ab/libdab_$L.so timeout -k 10 200 python -u scripts/rig_pcg_run.py c5_rig_16x64 $F >> $O 2>&1 || exit 1
    done
  done
done
for L in cur mf3; do
  rm -rf gpurun_out/r05az_$L
  DAB_LIB=scripts/ab/libdab_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05az_$L -o run --output-format csv -- python3 scripts/rig_pcg_run.py c5_rig_16x64 0 > /dev/null 2>&1 || exit 1
  echo "stats lib=$L" >> $O
  grep -h "k_mf_diag_frame" $(find gpurun_out/r05az_$L -name "*kernel_stats.csv") >> $O
done
