#!/bin/bash
# round 6: k_s_blocks with the last pairs of a block batched (masked exact +0.0 adds), U = 4
# and U = 8 pairs per group per step, against the unbatched remainder loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for L in base9 new sb8; do
    if [ $L = new ]; then X=; else X=scripts/ab/libdab_$L.so; fi
    DAB_LIB=$X timeout -k 10 180 python3 scripts/explicit_run.py c3_1kcam >> $O/c3.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
  done
done
cat $O/c3.jsonl | python3 -c "
import json,sys
rows=[json.loads(l) for l in sys.stdin]
for r in rows: print(r['lib'], round(r['iter_ms_median'],3), r['final_cost'])
print('costs identical across libraries:', len(set(tuple(r['costs']) for r in rows))==1)"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/explicit_run.py c3_1kcam > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h -E "k_s_blocks|k_s_zero|k_s_scatter|fillBuffer|k_s_diag" $O/prof/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_full_size.py tests/test_gpu_parity.py tests/test_gpu_dist.py -k "explicit or cholesky or c4" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
