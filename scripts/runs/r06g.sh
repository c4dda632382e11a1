#!/bin/bash
# round 6: config 1's first solve — the set-up's phases with the slab allocator on and off,
# and an API trace (hipMalloc, copies, syncs) of the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_default.txt 2>&1 || { tail $O/c1_default.txt; exit 1; }
DAB_DEV_SLAB=1 DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_slab.txt 2>&1 || { tail $O/c1_slab.txt; exit 1; }
grep "^rep" $O/c1_default.txt $O/c1_slab.txt
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 scripts/c1_first.py > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
ls -R $O/trace | head
