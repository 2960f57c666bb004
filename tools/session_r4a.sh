#!/bin/bash
# Round-4 GPU session: structured-buffer semantics probe, then the level-3/4 kernel A/B
# (k_bu_full + dskip vs k_bu_full vs round-3 k_bu_narrow; flat vs structured-buffer rows when the
# >4 GiB check passed), then the whole GPU suite.
set -u
mkdir -p gpurun_out
timeout -k 5 60 tools/ubench/bin/sbuf_check > gpurun_out/sbuf_check.log 2>&1
echo "sbuf_check rc=$?"; cat gpurun_out/sbuf_check.log
A=("all:-:--steps 10 --warmup 3" "full:MSBFS_TUNE=dskip=0:--steps 10 --warmup 3"
   "old:MSBFS_TUNE=full=0:--steps 10 --warmup 3")
tools/ab.sh "${A[@]}" || exit $?
if grep -q "check 3 (index \* stride beyond 4 GiB): ok" gpurun_out/sbuf_check.log; then
  bash tools/ab_lib.sh "sbuf:exp_lib/sbuf/libmsbfs.so:--steps 10 --warmup 3" || exit $?
fi
tools/ab.sh "${A[@]}" || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/pt_all.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/pt_all.log
