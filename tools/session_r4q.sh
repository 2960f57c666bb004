#!/bin/bash
# Round-4 GPU session q: kernel timelines of the 128-group (8-way round-robin rank) and RMAT-22 /
# 64-group steps, and of phase A / phase C in the 8-rank emulation, on the final round-4 code.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh prof128 prof22 profhc
