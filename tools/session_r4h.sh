#!/bin/bash
# Round-4 GPU session h: the tiled first pull with 256-thread blocks and global hub probes
# (tiles_bt=256, 4 or 5 blocks per CU) and the tail push after the tiles (push_after=1):
# oracle test, then A/B against the default.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "tiled_first_pull" > gpurun_out/pt_bt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_bt.log; [ $rc -eq 0 ] || exit 1
tools/ab.sh "b0:-:--steps 10 --warmup 3" "pa:MSBFS_TUNE=push_after=1:--steps 10 --warmup 3" \
  "b5:MSBFS_TUNE=tiles_bt=256:--steps 10 --warmup 3" \
  "b4:MSBFS_TUNE=tiles_bt=256;tiles_bpc=4:--steps 10 --warmup 3" "b0b:-:--steps 10 --warmup 3" \
  "pab:MSBFS_TUNE=push_after=1:--steps 10 --warmup 3" || exit $?
