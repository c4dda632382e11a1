#!/bin/bash
# PMC of the Cholesky's bulk update (k_syrk_big) at n = 5994: MFMA busy, LDS, waits
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
for pass in A B; do
  if [ $pass = A ]; then C=$PA; else C=$PB; fi
  rm -rf gpurun_out/r05al_$pass
  timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/r05al_$pass -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > gpurun_out/r05al_$pass.log 2>&1
  rc=$?; echo "pass $pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_mix.py k_syrk_big gpurun_out/r05al_A gpurun_out/r05al_B
python3 scripts/pmc_mix.py k_syrk_mfma gpurun_out/r05al_A gpurun_out/r05al_B
