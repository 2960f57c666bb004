#!/bin/bash
# Round-4 GPU session am: road grid, 256 groups (1655 ms now, 1558 in round 2) under the top-down
# batch tunings.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
G="python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 256 --steps 2"
for cfg in "d:MSBFS_X=0" "nobm:MSBFS_TUNE=td_bm=1099511627776" "bm16k:MSBFS_TUNE=td_bm=16384" \
           "nofused:MSBFS_TUNE=td_fused=0" "b16:MSBFS_TUNE=batch=16"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 $G > gpurun_out/gm_$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"ms": [0-9.]*' gpurun_out/gm_$name.log)"
done
