#!/bin/bash
# Round-4 GPU session ap: does an RCCL copy kernel started per piece (one-rank all-to-all of the
# piece's size) slow phase A's tiles? 8 ranks emulated, with and without.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 --no-roundrobin \
  > gpurun_out/hs_np.log 2>&1 || exit $?
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 --no-roundrobin \
  --rccl-pieces > gpurun_out/hs_rp.log 2>&1 || exit $?
for f in hs_np hs_rp; do
  echo "$f $(grep -o '"phase_a_ms_max": [0-9.]*\|"phase_a_wall_ms_max": [0-9.]*\|"correct": [a-z]*' gpurun_out/$f.log | tr '\n' ' ')"
  grep -o '"pieces_ms": [^]]*\]' gpurun_out/$f.log | head -1
done
