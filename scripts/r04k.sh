# Cholesky lookahead group A/B (n = 5994), first-solve / handle timing of config 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in "" "DAB_CHOL_GROUP=3" "DAB_CHOL_GROUP=4" "DAB_CHOL_NOGRAPH=1" "DAB_CHOL_GROUP=4 DAB_CHOL_BULK_GRID=512"; do
  echo "== $v"; env $v timeout -k 10 120 python -u scripts/chol_bench.py 5994 || exit $?
done > gpurun_out/chol_r04k.log 2>&1
cat gpurun_out/chol_r04k.log
DAB_SETUP_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 1 > gpurun_out/c1_r04k.log 2>&1 || exit $?
grep -E 'solve prep|iteration 0|create_ms|wall_ms' gpurun_out/c1_r04k.log | tail -40
