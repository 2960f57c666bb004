#!/bin/bash
# A/B of the level-2 push -> pull threshold (MSBFS_GAMMA2) over few-group RMAT-26/30, RMAT-22 and
# uniform graphs (round 2: chose gamma2 = 0.25). Run on the GPU box: bash tools/gamma_exp.sh
set -u
mkdir -p gpurun_out
run() { # name env args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 "$@" > gpurun_out/g_$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"dirs": "[A-Z]*"\|"ms": [0-9.]*' gpurun_out/g_$name.log | tr '\n' ' ')"
  [ $rc -le 1 ] || exit $rc
}
for g in 4 8 16; do
  run r26g${g}_d MSBFS_X=0 python bench.py --groups $g --steps 3 --warmup 1
  run r26g${g}_q MSBFS_GAMMA2=0.25 python bench.py --groups $g --steps 3 --warmup 1
  run r26g${g}_h MSBFS_GAMMA2=0.5 python bench.py --groups $g --steps 3 --warmup 1
done
run r22_d MSBFS_X=0 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1
run r22_q MSBFS_GAMMA2=0.25 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1
run uni_d MSBFS_X=0 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 2
run uni_q MSBFS_GAMMA2=0.25 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 2
run uni_h MSBFS_GAMMA2=0.5 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 2
run r30g16_d MSBFS_X=0 python bench.py --scale 30 --groups 16 --steps 1 --warmup 1
run r30g16_q MSBFS_GAMMA2=0.25 python bench.py --scale 30 --groups 16 --steps 1 --warmup 1
run r30g32_h MSBFS_GAMMA2=0.5 python bench.py --scale 30 --groups 32 --steps 1 --warmup 1
