#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool has no box for it (nothing
# ran, nothing charged); any call that ran ends this script with its result.
#   tools/gpurun_wait.sh <timeout-seconds> '<command>'
for i in $(seq 1 ${WAIT_TRIES:-45}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$1" -- "$2" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient rc=None charged=0.0s\|status=transient rc=None charged=Nones"; then
    echo "[wait] no box (attempt $i), retrying in 60 s"
    sleep 60
    continue
  fi
  echo "$out" | tail -12
  exit $rc
done
echo "[wait] gave up"
exit 3
