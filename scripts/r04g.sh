# per-wave timelines (trace build) of the fused pass: base, tables from k_cam_tables, and
# the camera side without gathers or arithmetic
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in base tab both; do
  case $v in tab) export DAB_FUSED_TAB=1;; both) unset DAB_FUSED_TAB; export DAB_FUSED_GV=6;; *) :;; esac
  DAB_TRACE_PER_WAVE=1 timeout -k 10 120 python -u scripts/trace_fused.py c3_1kcam > gpurun_out/tl_$v.log 2>&1 || exit $?
done
unset DAB_FUSED_GV
head -14 gpurun_out/tl_base.log; head -14 gpurun_out/tl_tab.log; head -14 gpurun_out/tl_both.log
