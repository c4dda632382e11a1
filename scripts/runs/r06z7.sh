#!/bin/bash
# round 6: k_schur_tiles one LDS buffer (DAB_TILE_SINGLE=1) against two, on the bench's rig
# (C5 EXACT + PCG) and config-1 lines, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06z7; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="python3 bench.py --no-c2 --no-c4 --steps 20 --warmup 5"
for rep in 1 2; do
  for v in 0 1; do
    DAB_TILE_SINGLE=$v timeout -k 10 300 $B > $O/b${v}_$rep.json 2> $O/b${v}_$rep.err || { echo "bench $v failed"; tail $O/b${v}_$rep.err; exit 1; }
    python3 -c "
import json; b=json.load(open('$O/b${v}_$rep.json'))
print('single=$v rep $rep', {k: round(b[k],4) if isinstance(b[k], float) else b[k] for k in ['rig_lm_explicit_iter_ms_median','rig_lm_pcg_iter_ms_median','c1_gpu_lm_iter_ms_median','c1_gpu_first_solve_wall_ms','c1_pipeline_gpu_s','c1_gpu_final_cost','rig_lm_explicit_costs']})"
  done
done
