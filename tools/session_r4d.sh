#!/bin/bash
# Round-4 GPU session d: default build twice (+ dskip=0), kernel oracle suite, then session c.
set -u
mkdir -p gpurun_out
tools/ab.sh "d1:-:--steps 10 --warmup 3" "d0:MSBFS_TUNE=dskip=0:--steps 10 --warmup 3" \
  "d2:-:--steps 10 --warmup 3" || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_kern.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_kern.log; [ $rc -eq 0 ] || exit 1
bash tools/session_r4c.sh
