#!/bin/bash
# Round-4 GPU session b: A/B of the pull-level kernels (default = k_bu_full + lean-level dskip,
# dskip=0, round-3 k_bu_narrow), the kernel oracle suite, one kernel trace and the level-3/4
# counter passes of the default build.
set -u
mkdir -p gpurun_out
A=("all:-:--steps 10 --warmup 3" "full:MSBFS_TUNE=dskip=0:--steps 10 --warmup 3"
   "old:MSBFS_TUNE=full=0:--steps 10 --warmup 3")
tools/ab.sh "${A[@]}" || exit $?
tools/ab.sh "${A[@]}" || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_hybrid.py -m gpu > gpurun_out/pt_kern.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_kern.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_session.sh prof26 || exit $?
PMC_RE="k_bu_full|k_bu_first" bash tools/gpu_session.sh pmcregex
