# uninitialised-memory hunt: finite poison (values used, not just multiplied by zero)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
DAB_DEV_POISON=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_full_size.py -m gpu -k "c5_pcg" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04p_a.log 2>&1
echo "c5_pcg finite poison rc=$?"; tail -3 gpurun_out/pytest_r04p_a.log
DAB_DEV_POISON=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04p_b.log 2>&1
echo "parity finite poison rc=$?"; grep -E "^FAILED" gpurun_out/pytest_r04p_b.log | head -60; tail -2 gpurun_out/pytest_r04p_b.log
DAB_DEV_POISON=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04p_c.log 2>&1
echo "parity NaN poison rc=$?"; grep -E "^FAILED" gpurun_out/pytest_r04p_c.log | head -60; tail -2 gpurun_out/pytest_r04p_c.log
exit 0
