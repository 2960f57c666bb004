#!/bin/bash
# Round-4 GPU session l: the whole GPU suite and smoke on the round-4 defaults, the bench twice,
# one kernel trace and the HBM / pipeline counter passes of the level kernels.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh pytest smoke || exit $?
tools/ab.sh "l1:-:--steps 20 --warmup 5" "l2:-:--steps 20 --warmup 5" || exit $?
bash tools/gpu_session.sh prof26 pmchbm
