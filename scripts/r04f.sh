# A/B: fused pass building its camera tables vs reading k_cam_tables' output (in the step)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 4 base tab=DAB_FUSED_TAB=1 > gpurun_out/ab6.log 2>&1 || exit $?
cat gpurun_out/ab6.log
