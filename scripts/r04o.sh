# flow Cholesky with lookahead ordering (timeline), column-form factor16 restored for the launch
# schedule; stream / pinned caches (config-1 create/destroy); host compaction A/B test
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_host.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04o.log; [ $rc -eq 0 ] || exit $rc
for v in "" "DAB_CHOL_FLOW=1" ""; do echo "== $v"; env $v timeout -k 10 120 python -u scripts/chol_bench.py 5994 || exit $?; done > gpurun_out/chol_r04o.log 2>&1
cat gpurun_out/chol_r04o.log
DAB_CHOL_FLOW=1 DAB_CHOL_FLOW_STAMPS=1 timeout -k 10 120 python -u scripts/chol_bench.py 5994 > gpurun_out/chol_r04o_stamps.log 2>&1 || exit $?
tail -1 gpurun_out/chol_r04o_stamps.log
DAB_SETUP_TIMING=1 timeout -k 10 300 python -u scripts/c1_pipeline.py 2 > gpurun_out/c1_r04o.log 2>&1 || exit $?
grep -E "create |destroy|create_ms|wall_ms" gpurun_out/c1_r04o.log | tail -24
