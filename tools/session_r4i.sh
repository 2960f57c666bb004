#!/bin/bash
# Round-4 GPU session i: the whole GPU suite and smoke on the push-after default, the bench
# twice, and a kernel trace of one RMAT-26 step.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh pytest smoke || exit $?
tools/ab.sh "i1:-:--steps 20 --warmup 5" "i2:-:--steps 20 --warmup 5" || exit $?
bash tools/gpu_session.sh prof26
