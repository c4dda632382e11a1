#!/bin/bash
# round 6: config 1's first solve on a fresh handle — phase times and a kernel + HIP API
# trace (where the set-up's ~2.3 ms and the solve preparation go)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06z2; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_first.txt 2>&1 || { echo "c1_first failed"; tail $O/c1_first.txt; exit 1; }
grep "^rep" $O/c1_first.txt
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $O/trace -o c1 -- python3 scripts/c1_first.py > $O/trace.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $O/trace.log; find $O/trace -name "*.csv" | head; exit $rc
