#!/bin/bash
# Round-4 GPU session ak: hybrid emulation at 2 / 4 / 8 ranks on the final round-4 code.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 --chunks 8 \
  > gpurun_out/hs248_final.log 2>&1 || exit $?
grep -o '"ranks": [0-9]*\|"hybrid_est_ms": [0-9.]*\|"roundrobin_ms_max": [0-9.]*\|"phase_a_ms_max": [0-9.]*\|"phase_c_ms_max": [0-9.]*\|"exposed_ms": [0-9.]*\|"correct": [a-z]*\|"single_ms": [0-9.]*' gpurun_out/hs248_final.log | tr '\n' ' '; echo
