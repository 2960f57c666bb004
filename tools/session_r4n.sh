#!/bin/bash
# Round-4 GPU session n: kernel + hybrid oracle tests on the new defaults (two-pass chunks,
# push-after without done probes), the bench, one trace, the 8-rank emulation, then the RMAT-30
# per-rank load of config 5 (32 groups).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_hybrid.py -m gpu > gpurun_out/pt_kern.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_kern.log; [ $rc -eq 0 ] || exit 1
tools/ab.sh "n1:-:--steps 20 --warmup 5" "n2:-:--steps 20 --warmup 5" || exit $?
bash tools/gpu_session.sh prof26 || exit $?
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks 8 \
  > gpurun_out/hsn8.log 2>&1 || exit $?
echo "hsn8: $(grep -o '"phase_a_ms_max": [0-9.]*\|"phase_c_ms_max": [0-9.]*\|"a2a_exposed_ms_est": [0-9.]*\|"hybrid_est_ms": [0-9.]*' gpurun_out/hsn8.log | tr '\n' ' ')"
MSBFS_TRACE=1 timeout -k 10 900 python bench.py --scale 30 --groups 32 --steps 1 --warmup 1 \
  > gpurun_out/r30g32.log 2>&1
echo "r30g32 rc=$? $(grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/r30g32.log | tr '\n' ' ')"
