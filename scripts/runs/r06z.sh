#!/bin/bash
# Round-6 final record on the round's final library, in two calls (each within gpurun's
# 20-minute limit): PART=tests — the -m gpu suite and smoke; PART=prof — the profile set
# (PMC traffic + VALU, bench line, kernel stats) and k_eval_bal's instruction mix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06z}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log; exit $rc
fi
TAG=$T bash scripts/gpu_prof.sh || exit $?
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
rm -rf gpurun_out/${T}_mix
timeout -s KILL 120 rocprofv3 --pmc $MIX -d gpurun_out/${T}_mix -o run --output-format csv -- python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1 --steps 10 --warmup 2 > gpurun_out/${T}_mix.log 2>&1
rc=$?; echo "mix rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_mix.py k_eval_bal gpurun_out/${T}_mix | tee gpurun_out/${T}_mix.txt
