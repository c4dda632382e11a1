#!/bin/bash
# GPU box: kernel trace of the config-5 check (eval passes + LM iterations) for timeline
# analysis (scripts/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/c5trace -o run --output-format csv -- python3 scripts/c5_check.py > gpurun_out/c5trace.log 2>&1 || { tail -5 gpurun_out/c5trace.log; exit 1; }
tail -6 gpurun_out/c5trace.log
