# column-update grid cap A/B (n = 5994), with a correctness pass at the chosen caps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in "" "DAB_CHOL_COL_GRID=32" "DAB_CHOL_COL_GRID=48" "DAB_CHOL_COL_GRID=64" "" "DAB_CHOL_COL_GRID=24" "DAB_CHOL_COL_GRID=40"; do
  echo "== $v"; env $v timeout -k 10 120 python -u scripts/chol_bench.py 5994 || exit $?
done > gpurun_out/chol_r04s.log 2>&1
cat gpurun_out/chol_r04s.log
DAB_CHOL_COL_GRID=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04s.log 2>&1
echo "dense with cap 32 rc=$?"; tail -2 gpurun_out/pytest_r04s.log
