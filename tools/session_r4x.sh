#!/bin/bash
# Round-4 GPU session x: where the step time outside the levels goes (0.1 vs 0.7 ms between
# processes): HIP runtime + kernel trace of 5 timed steps, twice.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/rt$i -o run -- \
    python bench.py --steps 5 --warmup 2 --verify 0 > gpurun_out/rt$i.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/rt$i.log
done
ls -R gpurun_out/rt1 | head -20
