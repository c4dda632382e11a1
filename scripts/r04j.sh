# candidate-table reuse: full GPU suite, config-1 pipeline (with set-up phase timing), bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/pytest_r04j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04j.log; [ $rc -eq 0 ] || exit $rc
DAB_SETUP_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04j.log 2>&1 || exit $?
tail -40 gpurun_out/c1_r04j.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r04j.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r04j.log
