#!/bin/bash
# Round-4 GPU session ah: wide_few gated on graph size — its test, then RMAT-22 / 64 groups and
# RMAT-26 / 128 groups.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "wide_threshold" > gpurun_out/pt_ah.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_ah.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "r22:-:--scale 22 --groups 64 --steps 30" "r22b:-:--scale 22 --groups 64 --steps 30" \
  "g128:-:--groups 128 --steps 10"
