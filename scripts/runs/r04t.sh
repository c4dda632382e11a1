# host-side filter / reader changes: host GPU tests and the config-1 pipeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_host_io.py tests/test_gpu_reuse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04t.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r04t.log; [ $rc -eq 0 ] || exit $rc
DAB_READ_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 3 > gpurun_out/c1_r04t.log 2>&1 || exit $?
grep -E "wall_ms|^read |parse" gpurun_out/c1_r04t.log | tail -12
