#!/bin/bash
# pair-major chunk sizes (DAB_XCHUNK) on the C5 rig: k_eval_pair time per size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for x in ${XS:-2048 4096 8192}; do
  rm -rf gpurun_out/xc$x
  DAB_SETUP_TIMING=1 DAB_XCHUNK=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xc$x -o run --output-format csv -- python3 scripts/c5_check.py > gpurun_out/xc$x.log 2>&1 || { tail -5 gpurun_out/xc$x.log; exit 1; }
  grep "eval pass" gpurun_out/xc$x.log
done
