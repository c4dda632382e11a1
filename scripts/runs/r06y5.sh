#!/bin/bash
# round 6: k_eval_bal's frames with the camera chunk's (ext, intr) computed when the map is
# affine (one dependent load less before the frames), C3 and C2 against the previous library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06y5; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
V="base=LIB=scripts/ab/libdab_base10.so new"
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 5 $V > $O/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail $O/ab_c3.txt; exit 1; }
tail -3 $O/ab_c3.txt
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 5 $V > $O/ab_c2.txt 2>&1 || { echo "ab c2 failed"; tail $O/ab_c2.txt; exit 1; }
tail -3 $O/ab_c2.txt
grep -h "cost dev" $O/ab_c3.txt $O/ab_c2.txt | awk '{print $NF}' | sort | uniq -c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_size.py -k "fused or split or c3 or c2 or eval" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
