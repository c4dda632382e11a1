#!/bin/bash
# round 6: the new one-vs-two LDS buffer test for k_schur_tiles and the tiles/pair-table tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zs; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "schur_tiles" > $O/pytest.log 2>&1; rc=$?; tail -6 $O/pytest.log; exit $rc
