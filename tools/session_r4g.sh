#!/bin/bash
# Round-4 GPU session g: k_bu_lean (first_u 2 / 4) oracle tests, then 1-GPU A/B of the lean
# pass kernel and the phase-C lean level (lean_level=2) in the 8-rank emulation.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "done_rows_skipped" > gpurun_out/pt_lean.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_lean.log; [ $rc -eq 0 ] || exit 1
tools/ab.sh "u0:-:--steps 10 --warmup 3" "u2:MSBFS_TUNE=first_u=2:--steps 10 --warmup 3" \
  "u4:MSBFS_TUNE=first_u=4:--steps 10 --warmup 3" "u0b:-:--steps 10 --warmup 3" \
  "u2b:MSBFS_TUNE=first_u=2:--steps 10 --warmup 3" "u4b:MSBFS_TUNE=first_u=4:--steps 10 --warmup 3" \
  || exit $?
for t in "-" "lean_level=2" "lean_level=2;first_u=2" "first_u=4" "lean_level=2;first_u=4"; do
  tag=$(echo "$t" | tr '=;' '__')
  if [ "$t" = "-" ]; then envs=(); else envs=("MSBFS_TUNE=$t"); fi
  env "${envs[@]}" timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 \
    --no-roundrobin --chunks 8 > "gpurun_out/hs_$tag.log" 2>&1 || exit $?
  echo "$t: $(grep -o '"phase_c_ms_max": [0-9.]*\|"hybrid_est_ms": [0-9.]*' gpurun_out/hs_$tag.log | tr '\n' ' ')"
  python3 - "gpurun_out/hs_$tag.log" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{") and '"per_rank"' in line:
        d = json.loads(line)
        print("  phase C per rank:", [round(x["phase_c_ms"], 2) for x in d["per_rank"]])
EOF
done
