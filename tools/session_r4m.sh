#!/bin/bash
# Round-4 GPU session m: two-pass wide chunks (chunk2) and lane refill (refill) for the
# one-lane-per-vertex pulls: oracle tests, 1-GPU A/B, 128-group A/B, phase-C A/B.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "two_pass or lane_refill or tiled_first or done_rows" \
  > gpurun_out/pt_c2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_c2.log; [ $rc -eq 0 ] || exit 1
A="--steps 10 --warmup 3"
tools/ab.sh "m0:-:$A" "mc:MSBFS_TUNE=chunk2=1:$A" "m0b:-:$A" "mcb:MSBFS_TUNE=chunk2=1:$A" \
  "g0:-:$A --groups 128" "gr:MSBFS_TUNE=refill=1:$A --groups 128" \
  "grc:MSBFS_TUNE=refill=1;chunk2=1:$A --groups 128" "g0b:-:$A --groups 128" \
  "grb:MSBFS_TUNE=refill=1:$A --groups 128" || exit $?
for t in "-" "refill=1" "refill=1;chunk2=1"; do
  tag=$(echo "$t" | tr '=;' '__')
  if [ "$t" = "-" ]; then envs=(); else envs=("MSBFS_TUNE=$t"); fi
  env "${envs[@]}" timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 \
    --no-roundrobin --chunks 8 > "gpurun_out/hsm_$tag.log" 2>&1 || exit $?
  echo "$t: $(grep -o '"phase_c_ms_max": [0-9.]*\|"hybrid_est_ms": [0-9.]*' gpurun_out/hsm_$tag.log | tr '\n' ' ')"
done
