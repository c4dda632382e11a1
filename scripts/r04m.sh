# persistent dataflow Cholesky: correctness (small forced, dense sizes, schedules, full-size
# trajectories), then timing against the launch schedule; config-1 timing; C2 timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r04m_dense.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r04m_dense.log; [ $rc -eq 0 ] || exit $rc
for v in "" "DAB_CHOL_FLOW=1" "DAB_CHOL_FLOW=1 DAB_CHOL_FLOW_GA=32" "DAB_CHOL_FLOW=1 DAB_CHOL_FLOW_GA=96" "DAB_CHOL_FLOW=1 DAB_CHOL_FLOW_GA=128" "DAB_CHOL_FLOW=1 DAB_CHOL_GROUP=3"; do
  echo "== $v"; env $v timeout -k 10 120 python -u scripts/chol_bench.py 5994 || exit $?
done > gpurun_out/chol_r04m.log 2>&1
cat gpurun_out/chol_r04m.log
DAB_CHOL_FLOW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c3_explicit or c3_converge" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04m_c3flow.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04m_c3flow.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_reuse.py tests/test_gpu_host.py tests/test_host_io.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04m.log; [ $rc -eq 0 ] || exit $rc
DAB_SETUP_TIMING=1 DAB_READ_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04m.log 2>&1 || exit $?
grep -E "solve prep|create |destroy|create_ms|wall_ms|^read " gpurun_out/c1_r04m.log | tail -60
timeout -k 10 120 python -u scripts/trace_fused.py c2_100cam > gpurun_out/trace_c2_r04m.log 2>&1 || exit $?
cat gpurun_out/trace_c2_r04m.log
