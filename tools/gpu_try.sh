#!/bin/bash
# Local wrapper around gpurun: retries ONLY when no GPU box is free (gpurun exit status 3, nothing
# ran, nothing charged), every 120 s, at most GPU_TRY_MAX times. Any other status ends it.
#   tools/gpu_try.sh <timeout-seconds> '<command>'
set -u
limit=$1; shift
for i in $(seq 1 "${GPU_TRY_MAX:-12}"); do
  /usr/local/graft/bin/gpurun --timeout "$limit" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpu_try] no box free (attempt $i); waiting 120 s"
  sleep 120
done
exit 3
