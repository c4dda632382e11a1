#!/bin/bash
# k_eval_bal VALU mix per ablation side (DAB_EVAL_SIDE: 0 shipped, 3 frames + point tables only,
# 5 no point tables, 2 no point rows): where the non-loop VALU goes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
: > gpurun_out/r05aw_mix.txt
for S in 0 3 5 2; do
  rm -rf gpurun_out/r05aw_mix_s$S
  DAB_EVAL_SIDE=$S timeout -s KILL 120 rocprofv3 --pmc $MIX -d gpurun_out/r05aw_mix_s$S -o run --output-format csv -- python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1 --steps 10 --warmup 2 > gpurun_out/r05aw_mix_s$S.log 2>&1
  rc=$?; echo "side $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "side $S" >> gpurun_out/r05aw_mix.txt
  python3 scripts/pmc_mix.py k_eval_bal gpurun_out/r05aw_mix_s$S >> gpurun_out/r05aw_mix.txt
done
