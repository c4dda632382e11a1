#!/bin/bash
# Round 5: -m gpu suite, the suite under DAB_DEV_POISON=1, the 8-rank bench rehearsal on one
# GPU beside the N=1 bench, then the fused evaluation kernel's VALU instruction mix (PMC),
# whole launch and per side (DAB_EVAL_SPLIT=1: camera-side launch, then point-side launch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05b_pytest.log; [ $rc -eq 0 ] || exit $rc
DAB_DEV_POISON=1 timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05b_pytest_poison.log 2>&1
rc=$?; echo "poison pytest rc=$rc"; tail -3 gpurun_out/r05b_pytest_poison.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 --lm-iters 2 --no-cpu > gpurun_out/r05b_bench1.json 2> gpurun_out/r05b_bench1.err
rc=$?; echo "bench1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
DAB_BENCH_DEVICE=0 DAB_BENCH_HOST_COLLECTIVE=1 timeout -k 10 420 python -u bench.py --gpus 8 --steps 5 --warmup 2 --lm-iters 2 > gpurun_out/r05b_bench8.json 2> gpurun_out/r05b_bench8.err
rc=$?; echo "bench8 rc=$rc"; tail -2 gpurun_out/r05b_bench8.err; [ $rc -eq 0 ] || exit $rc
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
B="python3 bench.py --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1 --steps 10 --warmup 2"
for mode in fused split; do
  if [ $mode = split ]; then export DAB_EVAL_SPLIT=1; fi
  timeout -s KILL 120 rocprofv3 --pmc $MIX -d gpurun_out/r05b_mix_$mode -o run --output-format csv -- $B > gpurun_out/r05b_mix_$mode.log 2>&1
  rc=$?; echo "mix $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
