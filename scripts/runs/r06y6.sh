#!/bin/bash
# round 6: the fused column update's factor and panel tails as noinline functions (tails1),
# and that kernel held to two waves per SIMD (tails2: no spills, so it fits beside a bulk
# work-group), against the previous library: n = 5994, C3 EXPLICIT, bits, stamps, tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06y6; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for L in base10 tails1 tails2; do
    echo "LIB=$L" >> $O/chol.txt
    DAB_LIB=scripts/ab/libdab_$L.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
    DAB_LIB=scripts/ab/libdab_$L.so timeout -k 10 180 python3 scripts/explicit_run.py c3_1kcam >> $O/c3.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
for L in tails1 tails2; do
  DAB_LIB=scripts/ab/libdab_$L.so DAB_DUMP=$O/x_$L.npy timeout -k 10 120 python3 scripts/chol_bench.py 5994 >> $O/chol.txt 2>&1 || exit 1
  python3 -c "import numpy as np; a=np.load('scripts/ab/x_r06c.npy'); b=np.load('$O/x_$L.npy'); print('$L vs r06c bitwise equal:', bool((a==b).all()))" >> $O/chol.txt
done
grep -v "^$" $O/chol.txt
python3 -c "
import json
rows=[json.loads(l) for l in open('$O/c3.jsonl')]
for r in rows: print(r['lib'], round(r['iter_ms_median'],3))
print('costs identical:', len(set(tuple(r['costs']) for r in rows))==1)"
DAB_LIB=scripts/ab/libdab_stamps.so timeout -k 10 120 python3 scripts/chol_bench.py 5994 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
