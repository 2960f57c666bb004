#!/bin/bash
# Round-4 GPU session t: first-step size of the non-lean full pull (tuning step1) — 1024 groups
# (level 3, default = a whole 8-row step), 128 groups (W = 2, default one row), hybrid phase C.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab.sh "s1024:-:--steps 10" "s1024c4:MSBFS_TUNE=step1=4:--steps 10" \
  "s1024c2:MSBFS_TUNE=step1=2:--steps 10" "s1024d:-:--steps 10" \
  "s128:-:--groups 128 --steps 10" "s128c4:MSBFS_TUNE=step1=4:--groups 128 --steps 10" \
  "s128c2:MSBFS_TUNE=step1=2:--groups 128 --steps 10" || exit $?
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 \
  > gpurun_out/hs_t0.log 2>&1 || exit $?
MSBFS_TUNE=step1=2 timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 \
  > gpurun_out/hs_t2.log 2>&1 || exit $?
MSBFS_TUNE=step1=4 timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 \
  > gpurun_out/hs_t4.log 2>&1 || exit $?
for f in hs_t0 hs_t2 hs_t4; do
  echo "$f $(grep -o '"phase_c_ms_max": [0-9.]*\|"phase_c_ms": \[[^]]*\]\|"correct": [a-z]*' gpurun_out/$f.log | tr '\n' ' ')"
done
