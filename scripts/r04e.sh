# ablations of the fused pass's camera side: local gathers (2), no arithmetic (4), both (6);
# and the halves alone (DAB_EVAL_SPLIT launches side 2 then side 1: timed as one pass)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 base loc=DAB_FUSED_GV=2 noar=DAB_FUSED_GV=4 both=DAB_FUSED_GV=6 > gpurun_out/ab5.log 2>&1 || exit $?
cat gpurun_out/ab5.log
