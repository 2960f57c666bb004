#!/bin/bash
# Round-4 GPU session ai: the road grid with 256 groups and the uniform graph on the final code.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 256 --steps 2 \
  > gpurun_out/grid256.log 2>&1 || exit $?
echo "grid256 $(grep -o '"ms": [0-9.]*\|"teps": [0-9.e+]*' gpurun_out/grid256.log | tr '\n' ' ')"
timeout -k 10 300 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 \
  --steps 5 > gpurun_out/uni_final.log 2>&1 || exit $?
echo "uniform $(grep -o '"ms": [0-9.]*\|"teps": [0-9.e+]*' gpurun_out/uni_final.log | tr '\n' ' ')"
