#!/bin/bash
# Round 5, first GPU pass: the -m gpu suite on the new allocator (guard tests, config-1 full
# size), the suite once more under DAB_DEV_POISON=1, then the 8-rank bench rehearsal on one GPU
# (host-staged collectives) beside the N=1 bench with the same short settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r05a_pytest.log; [ $rc -eq 0 ] || exit $rc
DAB_DEV_POISON=1 timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05a_pytest_poison.log 2>&1
rc=$?; echo "poison pytest rc=$rc"; tail -4 gpurun_out/r05a_pytest_poison.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --lm-iters 2 --no-cpu > gpurun_out/r05a_bench1.json 2> gpurun_out/r05a_bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
DAB_BENCH_DEVICE=0 DAB_BENCH_HOST_COLLECTIVE=1 timeout -k 10 420 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lm-iters 2 > gpurun_out/r05a_bench8.json 2> gpurun_out/r05a_bench8.err
rc=$?; echo "bench8 rc=$rc"; tail -3 gpurun_out/r05a_bench8.err; exit $rc
