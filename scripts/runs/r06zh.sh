#!/bin/bash
# round 6, the final library: the -m gpu suite under DAB_DEV_POISON=1 (every block handed out
# filled with NaN bytes), then the 8-rank bench rehearsal on one GPU (eight processes,
# host-staged collectives) beside the N = 1 line of the same short settings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06zh}; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
DAB_DEV_POISON=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest_gpu_poison.log 2>&1
rc=$?; echo "poison pytest rc=$rc"; tail -2 $O/pytest_gpu_poison.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --lm-iters 2 --no-cpu > $O/bench1.json 2> $O/bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
DAB_BENCH_DEVICE=0 DAB_BENCH_HOST_COLLECTIVE=1 timeout -k 10 420 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lm-iters 2 > $O/bench8.json 2> $O/bench8.err
rc=$?; echo "bench8 rc=$rc"; tail -2 $O/bench8.err; exit $rc
