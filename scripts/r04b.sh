# A/B: fused camera gathers per lane vs lane pairs (+ PMC of the pair variant)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 3 base gv1=DAB_FUSED_GV=1 gv2=DAB_FUSED_GV=2 r124=DAB_EVAL_ROLES=1,DAB_ROLES_V=124 > gpurun_out/ab2.log 2>&1 || exit $?
tail -6 gpurun_out/ab2.log
S1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"
S2="TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum"
S4="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES"
S6="TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_SPI_STALL_sum"
DAB_FUSED_GV=1 TAG=pmc_gv1 FILTER=k_eval bash scripts/pmc_sets.sh "$S1" "$S2" "$S4" "$S6" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_gv1.txt 2>&1 || exit $?
TAG=pmc_gv0 FILTER=k_eval bash scripts/pmc_sets.sh "$S6" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_gv0.txt 2>&1 || exit $?
cat gpurun_out/pmc_gv1.txt gpurun_out/pmc_gv0.txt
