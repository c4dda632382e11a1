#!/bin/bash
# the fused-eval edge-shape parity test, then the whole -m gpu suite under DAB_DEV_POISON=1
# on the round's final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "edge_shapes" --timeout 120 --timeout-method thread > gpurun_out/r05ac_edge.log 2>&1
rc=$?; echo "edge rc=$rc"; tail -6 gpurun_out/r05ac_edge.log; [ $rc -eq 0 ] || exit $rc
DAB_DEV_POISON=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05ac_pytest_poison.log 2>&1
rc=$?; echo "poison rc=$rc"; tail -3 gpurun_out/r05ac_pytest_poison.log; exit $rc
