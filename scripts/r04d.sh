# A/B: fused pass with / without the per-XCD L2 warm-up of the point array
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/eval_ab.py c3_1kcam 4 base warm=DAB_FUSED_GV=1 > gpurun_out/ab4.log 2>&1 || exit $?
cat gpurun_out/ab4.log
S3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
S1="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"
DAB_FUSED_GV=1 TAG=pmc_warm FILTER=k_eval bash scripts/pmc_sets.sh "$S1" "$S3" -- python3 scripts/eval_driver.py c3_1kcam 30 > gpurun_out/pmc_warm.txt 2>&1 || exit $?
cat gpurun_out/pmc_warm.txt
