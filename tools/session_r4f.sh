#!/bin/bash
# Round-4 GPU session f: hybrid emulation with the last-range-first pieces (chunks 4 and 8),
# then kernel timelines of phase A (rank 0) and phase C (ranks 0, 1).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for c in 4 8; do
  timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks $c \
    > gpurun_out/hybsim8_f$c.log 2>&1 || exit $?
  grep -o '"hybrid_est_ms": [0-9.]*\|"a2a_exposed_ms_est": [0-9.]*\|"phase_[ac]_ms_max": [0-9.]*' \
    gpurun_out/hybsim8_f$c.log | tr '\n' ' '; echo
done
bash tools/gpu_session.sh profhc
