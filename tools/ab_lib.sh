#!/bin/bash
# A/B of native library builds on the GPU box: for each "label:lib:bench args" run bench.py with
# MSBFS_LIB=lib (empty = the in-tree build) and print ms/step and the per-level ms.
#   bash tools/ab_lib.sh "base::--steps 10" "exp:exp_lib/x/libmsbfs.so:--steps 10"
set -u
mkdir -p gpurun_out
for cfg in "$@"; do
  IFS=: read -r label lib args <<< "$cfg"
  if [ -n "$lib" ]; then
    MSBFS_LIB=$PWD/$lib timeout -k 10 300 python bench.py $args > gpurun_out/ab_$label.log 2>&1
  else
    timeout -k 10 300 python bench.py $args > gpurun_out/ab_$label.log 2>&1
  fi
  rc=$?
  echo "== $label rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/ab_$label.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab_$label.log"; exit $rc; fi
done
