#!/bin/bash
# round 6: config 1's first solve with the staged upload and the slab allocator on by default
# (A/B against DAB_DEV_SLAB=0), then the set-up, guard and host tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06z3; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_first_$rep.txt 2>&1 || { echo "c1_first failed"; tail $O/c1_first_$rep.txt; exit 1; }
  DAB_DEV_SLAB=0 DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_first_noslab_$rep.txt 2>&1 || { echo "c1_first noslab failed"; exit 1; }
done
grep -H "^rep\|device: upload" $O/c1_first_*.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_setup.py tests/test_gpu_guard.py tests/test_gpu_host.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log; exit $rc
