#!/bin/bash
# round 6: the panel rows' solve right-looking (bitwise the same factor): panel micro, the
# n = 5994 factor + solve (bits against r06b's factor16-v2 solution), the Cholesky timeline;
# the split evaluation schedule's two launches before (round-5 library) and after
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 60 ./scripts/potrf_micro_1 > $O/potrf_micro.txt 2>&1 || { echo "potrf_micro failed"; cat $O/potrf_micro.txt; exit 1; }
head -14 $O/potrf_micro.txt
for rep in 1 2 3; do timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1; done
DAB_DUMP=$O/x.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06b_factor16v2.npy'); b=np.load('$O/x.npy'); print('right-looking panel solve vs r06b bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
cat $O/chol.txt
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/chol_trace -o run --output-format csv -- python3 scripts/chol_bench.py 5994 > $O/chol_trace.log 2>&1 || { echo "chol trace failed"; tail $O/chol_trace.log; exit 1; }
python3 scripts/chol_timeline.py $O/chol_trace 80 > $O/chol_timeline.txt 2>&1; sed -n 1,12p $O/chol_timeline.txt
for lib in r05 r06; do
  if [ $lib = r05 ]; then L=scripts/ab/libdab_r05.so; else L=; fi
  DAB_LIB=$L DAB_EVAL_SPLIT=1 timeout -k 10 180 rocprofv3 --kernel-trace -d $O/split_$lib -o run --output-format csv -- python3 scripts/eval_split_ab.py > $O/split_$lib.log 2>&1 || { echo "split $lib failed"; tail $O/split_$lib.log; exit 1; }
  python3 scripts/split_launch_times.py $O/split_$lib > $O/split_$lib.txt; echo "$lib:"; cat $O/split_$lib.txt
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_full_size.py \
  -k "dense or cholesky or c3_explicit or c5_explicit or c2_explicit or split_fused or lm_bal or lm_rig" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; exit $rc
