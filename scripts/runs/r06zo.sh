#!/bin/bash
# round 6: k_eval_bal camera frames built by the last point wave (before its table share) instead of camera wave 0, against the shipped library
# (base = libdab_base15.so), 6 interleaved reps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06zo; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base15.so pwframes"
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 6 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -3 $O/ab_c3.txt; grep "cost dev" $O/ab_c3.txt | awk '{print $NF}' | sort | uniq -c
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 6 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -3 $O/ab_c2.txt; grep "cost dev" $O/ab_c2.txt | awk '{print $NF}' | sort | uniq -c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_guard.py tests/test_gpu_dist.py -k "fused or split or c3 or c2 or eval or timeout or rccl or rank" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
