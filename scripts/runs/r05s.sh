#!/bin/bash
# A/B of the rig PCG preconditioner pass: k_mf_diag_rhs (DAB_MF_DIAG=0) vs k_mf_diag_frame (1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for f in 0 1 0 1; do
  rm -rf gpurun_out/r05s_$f
  DAB_MF_DIAG=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_$f -o run --output-format csv -- python3 scripts/rig_pcg_run.py > gpurun_out/r05s_$f.log 2>&1
  rc=$?; echo "form $f rc=$rc"; tail -1 gpurun_out/r05s_$f.log; [ $rc -eq 0 ] || exit $rc
  grep -h "k_mf_diag\|k_mf_frame<0>" $(find gpurun_out/r05s_$f -name "*kernel_stats.csv") | cut -c1-60,150-
done
