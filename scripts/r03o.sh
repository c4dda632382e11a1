#!/bin/bash
# rig pair-kernel point pre-gather A/B (DAB_PAIR_GATHER 1 | 0): rig eval + LM numbers from
# bench.py, kernel stats of the rig mixed PCG run, then the rig parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 1 0; do
  DAB_PAIR_GATHER=$g timeout -k 10 400 python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-c1 --steps 50 --warmup 5 > gpurun_out/bench_pg$g.json 2> gpurun_out/bench_pg$g.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_pg$g.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_pg$g.json'))
print('pair_gather=$g', {k: d.get(k) for k in ('rig_eval_ms_per_step','rig_eval_mobs_per_s','rig_pair_kernel_ms','rig_pair_kernel_roofline_frac','rig_lm_pcg_iter_ms_median','rig_lm_explicit_iter_ms_median','rig_lm_linear_iterations')})"
done
rm -rf gpurun_out/pgprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pgprof -o run --output-format csv -- python3 scripts/rig_mixed.py 3 > gpurun_out/pgprof.log 2>&1 || exit 1
grep -E "mixed|fp64" gpurun_out/pgprof.log | grep -v W2026 | head -4
find gpurun_out/pgprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/pg_stats.csv \;
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/pg_stats.csv')):
    if 'pair' in r['Name'] or 'eval' in r['Name']:
        print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {r['Calls']:>5} x {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:60]}")
PY
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "rig or c5 or pair" > gpurun_out/pytest_pg.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_pg.log
