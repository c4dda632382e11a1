cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv -- python3 scripts/c5_check.py > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
tail -6 gpurun_out/c5prof.log
find gpurun_out/c5prof -name "*kernel_stats.csv" -exec head -30 {} \;
