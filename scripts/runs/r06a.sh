#!/bin/bash
# round 6: the split schedule without dead work, the release library refusing the eval
# ablations, the multi-rank timeout, rotations near pi, the 4-rank C3 P2P rehearsal; then
# the split pass's two launch times at C3 (kernel trace, DAB_EVAL_SPLIT=1 on one rank)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r06a
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_guard.py tests/test_gpu_parity.py \
  -k "guard or eval_pass or refuses or split_fused or fused_eval or near_pi or jacobian_kernel" \
  > $O/pytest1.log 2>&1
rc=$?; echo "pytest1 rc=$rc"; tail -4 $O/pytest1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread \
  tests/test_gpu_full_size.py tests/test_gpu_dist.py -k "two_ranks_p2p or c4" \
  > $O/pytest2.log 2>&1
rc=$?; echo "pytest2 rc=$rc"; tail -4 $O/pytest2.log; [ $rc -eq 0 ] || exit $rc
SHORT="--steps 64 --warmup 8 --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1"
DAB_EVAL_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/split -o run --output-format csv -- python3 bench.py $SHORT > $O/split.log 2>&1 || { echo "split trace failed"; tail -20 $O/split.log; exit 1; }
python3 scripts/split_launch_times.py $O/split | tee $O/split_times.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/single -o run --output-format csv -- python3 bench.py $SHORT > $O/single.log 2>&1 || { echo "single trace failed"; tail -20 $O/single.log; exit 1; }
python3 scripts/split_launch_times.py $O/single | tee $O/single_times.txt
# the 8-rank bench rehearsal on one GPU (eight processes, host-staged collectives) beside the
# N = 1 line of the same short settings: the c4_* costs must equal N = 1's bitwise
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --lm-iters 2 --no-cpu > $O/bench1.json 2> $O/bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
DAB_BENCH_DEVICE=0 DAB_BENCH_HOST_COLLECTIVE=1 timeout -k 10 420 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lm-iters 2 > $O/bench8.json 2> $O/bench8.err
rc=$?; echo "bench8 rc=$rc"; tail -2 $O/bench8.err; exit $rc
