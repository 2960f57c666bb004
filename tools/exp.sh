#!/bin/bash
# Ad-hoc GPU experiment runner: each argument is "name|ENV=V ENV2=V|command args", run with its
# own time limit (EXP_LIMIT, default 600 s); stops at the first fault/abort/timeout (status > 1).
#   tools/exp.sh "t256|MSBFS_TRACE=1|python bench.py --steps 2 --warmup 0" ...
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  IFS='|' read -r name envs cmd <<< "$spec"
  echo "== $name: [$envs] $cmd"
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 "${EXP_LIMIT:-600}" $cmd > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  grep -h "level [1-4] \|\"metric\"" "gpurun_out/$name.log" | tail -n 5 | cut -c1-220
  if [ $rc -gt 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
done
