#!/bin/bash
# Round-4 GPU session an: level-3 done probes (tuning probe3) — 1024 / 128 groups, hybrid phase C.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu -k "done_rows or tiled_first" > gpurun_out/pt_an.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_an.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh "g1024:-:--steps 10" "g1024p:MSBFS_TUNE=probe3=1:--steps 10" \
  "g128:-:--groups 128 --steps 10" "g128p:MSBFS_TUNE=probe3=1:--groups 128 --steps 10" || exit $?
for t in 0 1; do
  MSBFS_TUNE=probe3=$t timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --chunks 8 \
    > gpurun_out/hs_p$t.log 2>&1 || exit $?
  echo "probe3=$t $(grep -o '"phase_c_ms_max": [0-9.]*\|"correct": [a-z]*' gpurun_out/hs_p$t.log | tr '\n' ' ')"
done
