#!/bin/bash
# round 6 (second pass, static first pieces, part-major order): k_eval_bal camera side as pieces claimed in order by every wave (the point waves
# join after their slices), pieces per work-group 8/16/24/32, C3 and C2 against the round-6
# library (scripts/ab/libdab_base11.so); then the evaluation parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06z5; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base11.so p16 p8=DAB_EVAL_PIECES=8 p12=DAB_EVAL_PIECES=12 p24=DAB_EVAL_PIECES=24"
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 3 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -6 $O/ab_c3.txt
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 3 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -6 $O/ab_c2.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_guard.py -k "fused or split or c3 or c2 or eval or timeout" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
