#!/bin/bash
# Round-4 GPU session al: per-group cumulative counters only with hskip — kernel tests, the road
# grid at 256 / 64 groups, the 1-GPU bench, then the hybrid emulation at 2 / 4 / 8 ranks.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_al.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_al.log; [ $rc -eq 0 ] || exit 1
for g in 256 64; do
  timeout -k 10 400 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups $g --steps 2 \
    > gpurun_out/grid_al$g.log 2>&1 || exit $?
  echo "grid$g $(grep -o '"ms": [0-9.]*' gpurun_out/grid_al$g.log)"
done
bash tools/ab.sh "g1024:-:--steps 20 --warmup 5" || exit $?
bash tools/session_r4ak.sh
