#!/bin/bash
# A/B of tuning settings on the GPU box: for each "label=spec" run bench.py (MSBFS_TUNE=spec,
# "-" for the defaults) and print ms/step and the per-level ms; stops at the first failure.
#   bash tools/ab_tune.sh "base=-" "e1=exp=1" -- --steps 10 --warmup 3 --verify 4
set -u
mkdir -p gpurun_out
specs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do specs+=("$1"); shift; done
[ $# -gt 0 ] && shift
for sp in "${specs[@]}"; do
  label=${sp%%=*}; tune=${sp#*=}
  if [ "$tune" = "-" ]; then
    timeout -k 10 300 python bench.py "$@" > "gpurun_out/ab_$label.log" 2>&1
  else
    MSBFS_TUNE="$tune" timeout -k 10 300 python bench.py "$@" > "gpurun_out/ab_$label.log" 2>&1
  fi
  rc=$?
  echo "== $label ($tune) rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/ab_$label.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab_$label.log"; exit $rc; fi
done
