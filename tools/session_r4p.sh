#!/bin/bash
# Round-4 GPU session p: profile refresh on the round-4 code — 128 groups (the 8-way round-robin
# rank), RMAT-22 / 64 groups (config 2), the road-like grid (config 4 proxy, 64 and 16 groups),
# and the tiled level's counters.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_session.sh prof128 prof22 rmat22 road road16 || exit $?
PMC_RE="k_pfx_tiles|k_push_tail_after" bash tools/gpu_session.sh pmcregex
