#!/bin/bash
# Round-4 GPU session y: step time outside the levels (tools/step_split.py), three processes.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  timeout -k 10 300 python tools/step_split.py > gpurun_out/split$i.log 2>&1 || exit $?
  tail -1 gpurun_out/split$i.log
done
