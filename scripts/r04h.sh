# full -m gpu suite (one process) + the config-1 pipeline breakdown
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_r04h.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r04h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/c1_pipeline.py 3 > gpurun_out/c1_r04h.log 2>&1 || exit $?
cat gpurun_out/c1_r04h.log
