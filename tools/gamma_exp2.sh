#!/bin/bash
# Follow-up to gamma_exp.sh with the new default: bit-parallel vs distance BFS for 1-3 groups
# (sets kAutoDistMaxGroups) and the headline / RMAT-30 configs for regressions.
set -u
mkdir -p gpurun_out
run() { # name env args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 "$@" > gpurun_out/g_$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"dirs": "[A-Z]*"\|"ms": [0-9.]*' gpurun_out/g_$name.log | tr '\n' ' ')"
  [ $rc -le 1 ] || exit $rc
}
for g in 1 2 3; do
  run r26g${g}_bp MSBFS_X=0 python bench.py --groups $g --steps 3 --warmup 1 --algo bitpar
  run r26g${g}_dist MSBFS_X=0 python bench.py --groups $g --steps 3 --warmup 1 --algo dist
done
run r26 MSBFS_X=0 python bench.py --steps 10 --warmup 2
run r26g128 MSBFS_X=0 python bench.py --groups 128 --steps 5 --warmup 1
run r30g256 MSBFS_X=0 python bench.py --scale 30 --groups 256 --steps 1 --warmup 1
run r30g32 MSBFS_X=0 python bench.py --scale 30 --groups 32 --steps 1 --warmup 1
