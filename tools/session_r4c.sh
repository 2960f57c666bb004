#!/bin/bash
# Round-4 GPU session c: the hybrid emulation with and without the overlapped exchange (8 ranks,
# then 2/4/8 with round robin) and the file-input preprocessing (device CSR build vs host build).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks 1 \
  > gpurun_out/hybsim8_c1.log 2>&1 || exit $?
tail -c 600 gpurun_out/hybsim8_c1.log | tr ',' '\n' | grep -E "hybrid_est|a2a_exposed|phase_[ac]_ms_max"
timeout -k 10 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin --chunks 4 \
  > gpurun_out/hybsim8_c4.log 2>&1 || exit $?
tail -c 600 gpurun_out/hybsim8_c4.log | tr ',' '\n' | grep -E "hybrid_est|a2a_exposed|phase_[ac]_ms_max"
timeout -k 10 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 --chunks 4 \
  > gpurun_out/hybsim248.log 2>&1 || exit $?
grep -o '"ranks": [0-9]*\|"hybrid_est_ms": [0-9.]*\|"roundrobin_ms_max": [0-9.]*' gpurun_out/hybsim248.log | tr '\n' ' '; echo
timeout -k 10 900 python tools/file_prep.py --scale 26 --groups 1024 --dir "${TMPDIR:-/tmp}/msbfs_fp" \
  > gpurun_out/file_prep.log 2>&1
echo "file_prep rc=$?"; tail -3 gpurun_out/file_prep.log
