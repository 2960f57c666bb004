#!/bin/bash
# Round-4 GPU session e: the hybrid emulation with pieces split by tile count and phase-C level
# traces (8 ranks, chunks 1 and 4).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks 4 \
  > gpurun_out/hybsim8_e4.log 2>&1 || exit $?
tail -c 600 gpurun_out/hybsim8_e4.log | tr ',' '\n' | grep -E "hybrid_est|a2a_exposed|phase_[ac]_ms_max"
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks 8 \
  > gpurun_out/hybsim8_e8.log 2>&1 || exit $?
tail -c 600 gpurun_out/hybsim8_e8.log | tr ',' '\n' | grep -E "hybrid_est|a2a_exposed|phase_[ac]_ms_max"
