cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "list rc=$?"
S1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"
S2="TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TD_TD_BUSY_sum"
S3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
S4="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES"
S5="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
TAG=pmc_fused FILTER=k_eval bash scripts/pmc_sets.sh "$S1" "$S2" "$S3" "$S4" "$S5" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_fused.txt 2>&1 || exit $?
DAB_EVAL_ROLES=1 TAG=pmc_roles FILTER=k_eval bash scripts/pmc_sets.sh "$S1" "$S2" "$S3" "$S4" "$S5" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_roles.txt 2>&1 || exit $?
cat gpurun_out/pmc_fused.txt gpurun_out/pmc_roles.txt
