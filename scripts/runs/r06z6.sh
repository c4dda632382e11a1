#!/bin/bash
# round 6: k_schur_tiles with one LDS buffer (batches of up to 64 points instead of ~34, each
# batch's DMA waited for) against the two-buffer schedule, C5 EXACT step (5 LM iterations,
# interleaved), kernel times under rocprofv3; then the explicit-step tests with the knob on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06z6; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  timeout -k 10 120 python3 scripts/rig_explicit.py 5 >> $O/ab.txt 2>&1 || exit 1; echo "^ two buffers" >> $O/ab.txt
  DAB_TILE_SINGLE=1 timeout -k 10 120 python3 scripts/rig_explicit.py 5 >> $O/ab.txt 2>&1 || exit 1; echo "^ one buffer" >> $O/ab.txt
done
cat $O/ab.txt
for v in 0 1; do
  DAB_TILE_SINGLE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr$v -o run --output-format csv -- python3 scripts/rig_explicit.py 3 > $O/tr$v.log 2>&1 || exit 1
  f=$(find $O/tr$v -name "*kernel_stats.csv"); grep -E "k_schur" $f | cut -d, -f1-4
done
DAB_TILE_SINGLE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full_size.py tests/test_gpu_dense.py tests/test_gpu_parity.py -k "explicit or tiles or c5 or schur" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
