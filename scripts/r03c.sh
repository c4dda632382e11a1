#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_host.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_host.log; ok $rc || exit $rc
timeout -k 10 600 python -u bench.py --no-lm --no-rig --no-c4 --no-c2 --steps 50 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_c1.json').read().strip().splitlines()[-1])
print({k: v for k, v in d.items() if k.startswith('c1') or k in ('value','ms_per_step')})"; tail -3 gpurun_out/bench_c1.err; exit $rc
