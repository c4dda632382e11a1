#!/bin/bash
# k_mf_frame32 camera-sum ablations (DAB_MF32_ACC: 0 fp64 LDS atomics, 2 none, 3 int64 LDS
# atomics, 4 fp32 LDS atomics; 2-4 give wrong products: timing only) on the C5 mixed PCG.
# 3 and 4 need scripts/experiments/mf32_int64_fp32_atomics.patch applied (not in the product).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for a in 0 2 3 4; do
  rm -rf gpurun_out/acc$a
  DAB_MF32_ACC=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/acc$a -o run --output-format csv -- python3 scripts/rig_mixed_only.py 2 > gpurun_out/acc$a.log 2>&1 || { tail -5 gpurun_out/acc$a.log; exit 1; }
done
