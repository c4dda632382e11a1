# A/B: fused camera-gather cache policy (plain / nt / sc1 / both) + PMC of sc1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 base gv16=DAB_FUSED_GV=16 gv2=DAB_FUSED_GV=2 gv18=DAB_FUSED_GV=18 > gpurun_out/ab3.log 2>&1 || exit $?
cat gpurun_out/ab3.log
S1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"
S2="TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum"
S3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
DAB_FUSED_GV=16 TAG=pmc_gv16 FILTER=k_eval bash scripts/pmc_sets.sh "$S1" "$S2" "$S3" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_gv16.txt 2>&1 || exit $?
cat gpurun_out/pmc_gv16.txt
