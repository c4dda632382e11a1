cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/eval_sweep.py ${SWEEP_CFG:-c3_1kcam} > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
cat gpurun_out/sweep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep_prof -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/sweep_prof.log 2>&1 || exit 1
find gpurun_out/sweep_prof -name "*kernel_stats.csv" -exec head -40 {} \;
