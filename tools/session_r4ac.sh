#!/bin/bash
# Round-4 GPU session ac: final-state check — every GPU test, smoke(), the 1-GPU bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh pytest smoke bench26
