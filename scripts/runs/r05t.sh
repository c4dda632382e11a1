#!/bin/bash
# PMC of the rig PCG preconditioner pass, both forms (DAB_MF_DIAG=0 / 1), two counter passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
for f in 0 1; do
  for pass in A B; do
    if [ $pass = A ]; then C=$PA; else C=$PB; fi
    rm -rf gpurun_out/r05t_${f}_$pass
    DAB_MF_DIAG=$f timeout -s KILL 150 rocprofv3 --pmc $C -d gpurun_out/r05t_${f}_$pass -o run --output-format csv -- python3 scripts/rig_pcg_run.py > gpurun_out/r05t_${f}_$pass.log 2>&1
    rc=$?; echo "form $f pass $pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_mix.py k_mf_diag gpurun_out/r05t_0_A gpurun_out/r05t_0_B gpurun_out/r05t_1_A gpurun_out/r05t_1_B
