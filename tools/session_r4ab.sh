#!/bin/bash
# Round-4 GPU session ab: two-pass hub chunks with early exit on the prefix level 2 of passes
# without tiles (tuning chunk2_l2) — test, then A/B at 64 / 128 / 256 groups.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "two_pass" > gpurun_out/pt_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_ab.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "g128:-:--groups 128 --steps 10" "g128c:MSBFS_TUNE=chunk2_l2=1:--groups 128 --steps 10" \
  "g256:-:--groups 256 --steps 10" "g256c:MSBFS_TUNE=chunk2_l2=1:--groups 256 --steps 10" \
  "g64:-:--groups 64 --steps 10" "g64c:MSBFS_TUNE=chunk2_l2=1:--groups 64 --steps 10" \
  "g128cw:MSBFS_TUNE=chunk2_l2=1,wide_few=32:--groups 128 --steps 10"
