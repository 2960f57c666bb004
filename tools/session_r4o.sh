#!/bin/bash
# Round-4 GPU session o: uneven word split test, then the phase-C balance experiment with the
# uneven split (tools/hybrid_balance.py), and the hybrid emulation at 2 / 4 / 8 ranks.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_hybrid.py -m gpu -k "uneven" > gpurun_out/pt_uneven.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt_uneven.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python tools/hybrid_balance.py --scale 26 --ranks 8 \
  --orders orig cluster uneven > gpurun_out/balance4.log 2>&1 || exit $?
cut -c1-400 gpurun_out/balance4.log
timeout -k 10 600 python tools/hybrid_balance.py --scale 26 --ranks 8 --orders uneven \
  --uneven 3,2,2,2,2,2,2,1 > gpurun_out/balance4b.log 2>&1 || exit $?
timeout -k 10 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 --chunks 8 \
  > gpurun_out/hs248.log 2>&1 || exit $?
grep -o '"ranks": [0-9]*\|"hybrid_est_ms": [0-9.]*\|"roundrobin_ms_max": [0-9.]*\|"phase_c_ms_max": [0-9.]*' gpurun_out/hs248.log | tr '\n' ' '; echo
