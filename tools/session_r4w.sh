#!/bin/bash
# Round-4 GPU session w: k_pfx_tiles counter slices (5 / 6) and epilogue passes in flight (1 / 2),
# library builds A/B at 1024 groups.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab_lib.sh "base::--steps 10" "s6:exp_lib/s6/libmsbfs.so:--steps 10" \
  "nh2:exp_lib/nh2/libmsbfs.so:--steps 10" "s6nh2:exp_lib/s6nh2/libmsbfs.so:--steps 10" \
  "base2::--steps 10" "s62:exp_lib/s6/libmsbfs.so:--steps 10" \
  "nh22:exp_lib/nh2/libmsbfs.so:--steps 10" "s6nh22:exp_lib/s6nh2/libmsbfs.so:--steps 10"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_cli_gpu.py -m gpu -k "spmd" > gpurun_out/pt_w.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_w.log; [ $rc -eq 0 ] || exit 1
