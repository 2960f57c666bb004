#!/bin/bash
# Round-4 GPU session ag: RMAT-22 / 64 groups with and without the wide_few threshold.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/ab.sh "r22:-:--scale 22 --groups 64 --steps 30" "r22w0:MSBFS_TUNE=wide_few=0:--scale 22 --groups 64 --steps 30" \
  "r22b:-:--scale 22 --groups 64 --steps 30" "r22w0b:MSBFS_TUNE=wide_few=0:--scale 22 --groups 64 --steps 30" \
  "r22w64:MSBFS_TUNE=wide_few=64:--scale 22 --groups 64 --steps 30"
