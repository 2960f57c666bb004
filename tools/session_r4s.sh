#!/bin/bash
# Round-4 GPU session s: kernel tests (incl. the first-pull wide threshold), then A/B of
# wide_few at 128 / 256 / 1024 groups.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_s.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_s.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "g128:-:--groups 128 --steps 10" "g128w0:MSBFS_TUNE=wide_few=0:--groups 128 --steps 10" \
  "g256:-:--groups 256 --steps 10" "g256w0:MSBFS_TUNE=wide_few=0:--groups 256 --steps 10" \
  "g1024:-:--steps 10" "g64:-:--groups 64 --steps 10" "g64w0:MSBFS_TUNE=wide_few=0:--groups 64 --steps 10"
