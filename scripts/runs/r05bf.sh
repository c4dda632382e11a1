#!/bin/bash
# the small-angle identity test of the table staging loads-first (rd_is_identity) in the rig
# kernels: rig parity tests, then C5 PCG / EXPLICIT against the round's record library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05bf.txt; : > $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_setup.py -k "rig or c5 or pair or small or mf or pcg" >> $O 2>&1 || { echo "pytest rc=$?" >> $O; exit 1; }
for r in 1 2; do
  for L in head new; do
    LIB=deeparc-sfm_amd/libdab.so; [ $L = head ] && LIB=scripts/ab/libdab_head.so
    for F in 0 1; do
      echo "lib=$L fp32=$F" >> $O
      DAB_LIB=$LIB timeout -k 10 200 python -u scripts/rig_pcg_run.py c5_rig_16x64 $F >> $O 2>&1 || exit 1
    done
  done
done
