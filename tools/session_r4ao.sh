#!/bin/bash
# Round-4 GPU session ao: the final in-tree build — kernel tests, smoke, bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh pytest_kernels smoke bench26
