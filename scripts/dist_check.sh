cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 scripts/dist_check.py --device 0 --host-collective > gpurun_out/dist_check.log 2>&1
rc=$?; echo "dist rc=$rc"; tail -40 gpurun_out/dist_check.log
[ $rc -eq 0 ] || exit $rc
DAB_BENCH_DEVICE=0 DAB_BENCH_HOST_COLLECTIVE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --lm-iters 3 > gpurun_out/bench_n2_rehearsal.log 2>&1
rc=$?; echo "bench n2 rc=$rc"; tail -3 gpurun_out/bench_n2_rehearsal.log; exit $rc
