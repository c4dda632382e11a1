#!/bin/bash
# round 6: factor16 rewritten (one 64-bit DPP per broadcast, the inverse carried along the
# factorisation, no AGPR spills): micro-benchmark of the 64x64 panel step both ways, the
# n = 5994 factor + solve A/B (round-5 factor16 in scripts/ab/libdab_f16v1.so), parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in 0 1 2; do timeout -k 10 60 ./scripts/potrf_micro_$v > $O/potrf_micro_$v.txt 2>&1 || { echo "potrf_micro_$v failed"; cat $O/potrf_micro_$v.txt; exit 1; }; done
head -14 $O/potrf_micro_0.txt $O/potrf_micro_1.txt $O/potrf_micro_2.txt
for rep in 1 2 3; do
  DAB_LIB=scripts/ab/libdab_f16v1.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol_ab.txt 2>&1 || exit 1
  echo "^ round-5 factor16" >> $O/chol_ab.txt
  timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol_ab.txt 2>&1 || exit 1
  echo "^ round-6 factor16" >> $O/chol_ab.txt
done
for rep in 1 2 3; do
  DAB_CHOL_BULK_DMA=1 timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol_ab.txt 2>&1 || exit 1
  echo "^ round-6 factor16 + LDS-DMA bulk (k_syrk_bigd)" >> $O/chol_ab.txt
done
DAB_CHOL_BULK_DMA=1 DAB_DUMP=$O/x_v3.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 > /dev/null 2>&1 || exit 1
DAB_LIB=scripts/ab/libdab_f16v1.so DAB_DUMP=$O/x_v1.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 > /dev/null 2>&1 || exit 1
DAB_DUMP=$O/x_v2.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 > /dev/null 2>&1 || exit 1
python3 -c "import numpy as np; a=np.load('$O/x_v1.npy'); b=np.load('$O/x_v2.npy'); c=np.load('$O/x_v3.npy'); print('factor16 v1 vs v2 bitwise equal:', bool((a==b).all()), 'max rel diff', float(abs(a-b).max()/abs(a).max())); print('bulk dma vs shipped bitwise equal:', bool((c==b).all()), 'max rel diff', float(abs(c-b).max()/abs(b).max()))" >> $O/chol_ab.txt
cat $O/chol_ab.txt
# config 1's first solve on a fresh handle, phase by phase (set-up and solve preparation)
DAB_SETUP_TIMING=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_first.txt 2>&1 || { echo "c1_first failed"; tail $O/c1_first.txt; exit 1; }
DAB_DEV_SLAB=1 timeout -k 10 120 python3 scripts/c1_first.py > $O/c1_first_slab.txt 2>&1 || { echo "c1_first slab failed"; exit 1; }
grep "^rep" $O/c1_first.txt $O/c1_first_slab.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_full_size.py \
  -k "dense or cholesky or c3_explicit or c5_explicit or c2_explicit or lm_bal or lm_rig" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log; exit $rc
