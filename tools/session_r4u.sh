#!/bin/bash
# Round-4 GPU session u: tiled first pull level at 4 words (tuning tiles_w=4) — tests, then A/B at
# 256 groups (W = 4) and per-level times at 512 groups (W = 8, tiles vs per-vertex pulls).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "tiled_first_pull" > gpurun_out/pt_u.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_u.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "g256:-:--groups 256 --steps 10" "g256t4:MSBFS_TUNE=tiles_w=4:--groups 256 --steps 10" \
  "g256t4pb:MSBFS_TUNE=tiles_w=4,push_after=0:--groups 256 --steps 10" \
  "g512:-:--groups 512 --steps 10" "g512t0:MSBFS_TUNE=tiles=0:--groups 512 --steps 10" \
  "g256b:-:--groups 256 --steps 10" "g256t4b:MSBFS_TUNE=tiles_w=4:--groups 256 --steps 10"
