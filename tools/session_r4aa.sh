#!/bin/bash
# Round-4 GPU session aa: small all-reduces through pinned buffers — bench / hybrid / distributed
# GPU tests; then the 128-group kernel timeline with wide_few.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_bench_gpu.py tests/test_hybrid.py tests/test_distributed.py -m gpu > gpurun_out/pt_aa.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_aa.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_session.sh prof128 || exit $?
