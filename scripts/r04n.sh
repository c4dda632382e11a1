# c5_pcg termination (slab allocator A/B), flow Cholesky timeline, config-1 timing, C2 timeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
DAB_DEV_SLAB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c5_pcg" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04n_a.log 2>&1
echo "c5_pcg slab on rc=$?"; tail -3 gpurun_out/pytest_r04n_a.log
DAB_DEV_SLAB=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c5_pcg" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04n_b.log 2>&1
echo "c5_pcg slab off rc=$?"; tail -3 gpurun_out/pytest_r04n_b.log
DAB_DEV_POISON=1 DAB_DEV_SLAB=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c5_pcg" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04n_c.log 2>&1
echo "c5_pcg poison, slab off rc=$?"; tail -3 gpurun_out/pytest_r04n_c.log
DAB_DEV_SLAB=1 DAB_DEV_GUARD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c5_pcg" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04n_d.log 2>&1
echo "c5_pcg guard rc=$?"; grep -E "dab guard" gpurun_out/pytest_r04n_d.log | head; tail -3 gpurun_out/pytest_r04n_d.log
DAB_DEV_POISON=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04n_e.log 2>&1
echo "parity poison rc=$?"; tail -8 gpurun_out/pytest_r04n_e.log
DAB_CHOL_FLOW=1 DAB_CHOL_FLOW_STAMPS=1 timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/chol_r04n.log 2>&1 || exit $?
tail -1 gpurun_out/chol_r04n.log
DAB_SETUP_TIMING=1 DAB_READ_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04n.log 2>&1 || exit $?
grep -E "solve prep|create |destroy|create_ms|wall_ms|^read " gpurun_out/c1_r04n.log | tail -60
timeout -k 10 120 python -u scripts/trace_fused.py c2_100cam > gpurun_out/trace_c2_r04n.log 2>&1 || exit $?
head -12 gpurun_out/trace_c2_r04n.log
