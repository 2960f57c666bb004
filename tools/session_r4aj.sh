#!/bin/bash
# Round-4 GPU session aj: uniform graph per-level records under a few tunings (lean pass, row
# skipping, unfiltered kernel) to find what made it slower than round 2 (27.2 ms).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
U="python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 5"
for cfg in "d:MSBFS_X=0" "nolean:MSBFS_TUNE=lean=0" "nodskip:MSBFS_TUNE=dskip=0" \
           "nofull:MSBFS_TUNE=full=0" "nochunk2:MSBFS_TUNE=chunk2=0" "lean4:MSBFS_TUNE=lean_level=4"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 $U --trace-out gpurun_out/uj_$name.json > gpurun_out/uj_$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"ms": [0-9.]*' gpurun_out/uj_$name.log) $(python -c "
import json,sys; t=json.load(open('gpurun_out/uj_$name.json')); print(' '.join(f\"{r['dir']}{r['ms']:.2f}\" for r in t))")"
done
