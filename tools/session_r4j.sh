#!/bin/bash
# Round-4 GPU session j: kernel oracle suite (lbits, dskip3, push_after variants), then A/B of
# the leader-combined done bits and the level-3 row skipping.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_kern.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_kern.log; [ $rc -eq 0 ] || exit 1
A="--steps 10 --warmup 3"
tools/ab.sh "j0:-:$A" "jl:MSBFS_TUNE=lbits=1:$A" "j3:MSBFS_TUNE=dskip3=1:$A" \
  "jl3:MSBFS_TUNE=lbits=1;dskip3=1:$A" "j0b:-:$A" "jlb:MSBFS_TUNE=lbits=1:$A" \
  "j3b:MSBFS_TUNE=dskip3=1:$A" "jl3b:MSBFS_TUNE=lbits=1;dskip3=1:$A" || exit $?
