# small-system Cholesky without graph, create/destroy phases, C2 per-wave timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_parity.py tests/test_gpu_reuse.py tests/test_gpu_host.py tests/test_host_io.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04l.log; [ $rc -eq 0 ] || exit $rc
DAB_SETUP_TIMING=1 DAB_READ_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04l.log 2>&1 || exit $?
grep -E "solve prep|create |destroy|create_ms|wall_ms|^read " gpurun_out/c1_r04l.log | tail -60
timeout -k 10 120 python -u scripts/chol_bench.py 5994 || exit $?
timeout -k 10 120 python -u scripts/trace_fused.py c2_100cam > gpurun_out/trace_c2_r04l.log 2>&1 || exit $?
cat gpurun_out/trace_c2_r04l.log
