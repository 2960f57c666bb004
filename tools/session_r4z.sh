#!/bin/bash
# Round-4 GPU session z: pinned staging of the batch sources — kernel tests, then the step split
# (outliers outside the level loop) in three processes and bench runs.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_z.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_z.log; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python tools/step_split.py --steps 60 > gpurun_out/splitz$i.log 2>&1 || exit $?
  tail -1 gpurun_out/splitz$i.log
done
bash tools/ab.sh "z1:-:--steps 20 --warmup 5" "z2:-:--steps 20 --warmup 5" "z3:-:--steps 20 --warmup 5"
