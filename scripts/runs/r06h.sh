#!/bin/bash
# round 6: config 1's LM iteration — k_schur_tiles' batches per work-group (DAB_TILE_MINB;
# 8 kept the partial sums small but gave C1's 313 batches only 39 work-groups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06h}; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  for m in 8 4 2; do
    echo "MINB=$m" >> $O/c1.txt
    DAB_TILE_MINB=$m timeout -k 10 120 python3 scripts/c1_first.py >> $O/c1.txt 2>&1 || exit 1
  done
done
grep -E "MINB|rep 2" $O/c1.txt
for m in 8 4 2; do
  DAB_TILE_MINB=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python3 scripts/c1_first.py > $O/prof_$m.log 2>&1 || exit 1
  echo "MINB=$m"; grep -h -E "schur_tiles|schur_sum_tiles|schur_y" $O/prof_$m/run_kernel_stats.csv | cut -d, -f1-5
done
