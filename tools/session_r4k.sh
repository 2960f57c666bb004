#!/bin/bash
# Round-4 GPU session k: kernel oracle suite with the hit-skip lean pass (hskip) and the
# hybrid tests, then A/B of hskip on RMAT-26 / 1024 groups and the 128-group load.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_hybrid.py -m gpu > gpurun_out/pt_kern.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_kern.log; [ $rc -eq 0 ] || exit 1
A="--steps 10 --warmup 3"
tools/ab.sh "k0:-:$A" "kh:MSBFS_TUNE=hskip=1:$A" "k0b:-:$A" "khb:MSBFS_TUNE=hskip=1:$A" \
  "k128:-:$A --groups 128" "kh128:MSBFS_TUNE=hskip=1:$A --groups 128" || exit $?
