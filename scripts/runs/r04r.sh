# CG partials overrun fixed: the suite with packed buffers (DAB_DEV_SLAB=1), then a guard pass
# (zero canaries) over parity + full size
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
DAB_DEV_SLAB=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04r_slab.log 2>&1
rc=$?; echo "slab suite rc=$rc"; grep -E "^FAILED" gpurun_out/pytest_r04r_slab.log | head; tail -2 gpurun_out/pytest_r04r_slab.log
DAB_DEV_GUARD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04r_guard.log 2>&1
echo "guard rc=$?"; grep -c "dab guard" gpurun_out/pytest_r04r_guard.log; grep "dab guard" gpurun_out/pytest_r04r_guard.log | sort | uniq -c | head -20; tail -2 gpurun_out/pytest_r04r_guard.log
DAB_DEV_SLAB=1 DAB_SETUP_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04r.log 2>&1 || exit $?
grep -E "destroy|create_ms|wall_ms" gpurun_out/c1_r04r.log | tail -12
