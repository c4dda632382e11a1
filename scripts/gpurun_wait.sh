#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free slot (nothing
# ran and nothing was charged); any call that actually ran is never repeated.
# usage: scripts/gpurun_wait.sh LOG TIMEOUT_S 'command'
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "run [1-9]" "$log"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
