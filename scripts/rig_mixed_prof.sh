#!/bin/bash
# kernel-trace breakdown of the C5 mixed-precision PCG (scripts/rig_mixed_only.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -rf gpurun_out/rmx
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rmx -o run --output-format csv -- python3 scripts/rig_mixed_only.py 5 > gpurun_out/rmx.log 2>&1 || { tail -5 gpurun_out/rmx.log; exit 1; }
grep "rep" gpurun_out/rmx.log
