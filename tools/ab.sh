#!/bin/bash
# Quick A/B timing on the GPU box: bench.py runs printing ms/step and per-level ms.
# usage: tools/ab.sh "<label>:<env>:<bench args>" ...   (env: VAR=x,VAR2=y or -)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  IFS=: read -r label envs args <<< "$spec"
  envcmd=()
  if [ "$envs" != "-" ]; then IFS=, read -ra envcmd <<< "$envs"; fi
  env "${envcmd[@]}" timeout -k 10 300 python bench.py $args > "gpurun_out/ab_$label.log" 2>&1
  rc=$?
  echo "$label rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/ab_$label.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab_$label.log"; exit $rc; fi
done
