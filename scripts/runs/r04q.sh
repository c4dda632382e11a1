# bank-spread R,t layout of the fused pass: parity, then A/B against the plain layout build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -m gpu -x -q -k "not c5" --timeout 200 --timeout-method thread > gpurun_out/pytest_r04q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/eval_ab.py c3_1kcam 4 pad plain=LIB=scripts/alt/libdab_rtpad0.so padtab=DAB_FUSED_TAB=1 plaintab=LIB=scripts/alt/libdab_rtpad0.so,DAB_FUSED_TAB=1 > gpurun_out/ab8.log 2>&1 || exit $?
tail -6 gpurun_out/ab8.log
timeout -k 10 300 python -u scripts/eval_ab.py c2_100cam 4 pad plain=LIB=scripts/alt/libdab_rtpad0.so > gpurun_out/ab9.log 2>&1 || exit $?
tail -4 gpurun_out/ab9.log
