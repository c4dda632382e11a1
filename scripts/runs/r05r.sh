#!/bin/bash
# k_eval_bal's VALU instruction mix at C3 (PMC, one pass: all counters fit the SQ block),
# whole launch and per side (DAB_EVAL_SPLIT=1), then the profile set (traffic, bench, stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
B="python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1 --steps 10 --warmup 2"
for mode in fused split; do
  rm -rf gpurun_out/r05r_mix_$mode
  if [ $mode = split ]; then export DAB_EVAL_SPLIT=1; fi
  timeout -s KILL 120 rocprofv3 --pmc $MIX -d gpurun_out/r05r_mix_$mode -o run --output-format csv -- $B > gpurun_out/r05r_mix_$mode.log 2>&1
  rc=$?; echo "mix $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
unset DAB_EVAL_SPLIT
python3 scripts/pmc_mix.py k_eval_bal gpurun_out/r05r_mix_fused gpurun_out/r05r_mix_split > gpurun_out/r05r_mix.txt
cat gpurun_out/r05r_mix.txt
TAG=r05r bash scripts/gpu_prof.sh
