#!/bin/bash
# Rodrigues series with SGPR constants (fma_sk): k_eval_bal A/B against the base library (C3, C2),
# and the VALU mix of the new library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05ax.txt; : > $O
timeout -k 10 240 python -u scripts/eval_ab.py c3_1kcam 4 base=LIB=scripts/ab/libdab_base.so new >> $O 2>&1 || { echo "ab c3 rc=$?" >> $O; exit 1; }
timeout -k 10 240 python -u scripts/eval_ab.py c2_100cam 4 base=LIB=scripts/ab/libdab_base.so new >> $O 2>&1 || { echo "ab c2 rc=$?" >> $O; exit 1; }
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
rm -rf gpurun_out/r05ax_mix
timeout -s KILL 120 rocprofv3 --pmc $MIX -d gpurun_out/r05ax_mix -o run --output-format csv -- python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1 --steps 10 --warmup 2 > gpurun_out/r05ax_mix.log 2>&1
rc=$?; echo "mix rc=$rc" >> $O; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_mix.py k_eval_bal gpurun_out/r05ax_mix >> $O
