#!/bin/bash
# Round-4 GPU session v: tile-local counters in k_pfx_tiles (default) and the pipelined variant
# (tiles_pipe=1: probes and code loads a round ahead) — tests, then A/B at 1024 / 512 groups.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "tiled or hybrid or done_rows" > gpurun_out/pt_v.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_v.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "d1024:-:--steps 10" "p1024:MSBFS_TUNE=tiles_pipe=1:--steps 10" \
  "d1024b:-:--steps 10" "p1024b:MSBFS_TUNE=tiles_pipe=1:--steps 10" \
  "d512:-:--groups 512 --steps 10" "p512:MSBFS_TUNE=tiles_pipe=1:--groups 512 --steps 10"
