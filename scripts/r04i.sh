# pooled allocator + reader: host/reuse/setup tests, config-1 pipeline breakdown; fused-pass
# camera prologue priority and wave-order A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_reuse.py tests/test_gpu_setup.py tests/test_host_io.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r04i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/c1_pipeline.py 4 > gpurun_out/c1_r04i.log 2>&1 || exit $?
cat gpurun_out/c1_r04i.log
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 base prio=DAB_FUSED_GV=8 old=DAB_FUSED_V=1000 > gpurun_out/ab7.log 2>&1 || exit $?
tail -4 gpurun_out/ab7.log
