#!/bin/bash
# Round-4 GPU session r: the first-pull wide threshold for few words (the round-robin ranks at
# 4 / 8 GPUs: 256 / 128 groups, no tiles), A/B of --wide-degree.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
A="--steps 10 --warmup 3 --verify 0"
tools/ab.sh "w128d32:-:$A --groups 128" "w128d128:-:$A --groups 128 --wide-degree 128" \
  "w128d512:-:$A --groups 128 --wide-degree 512" "w128d2k:-:$A --groups 128 --wide-degree 2048" \
  "w256d32:-:$A --groups 256" "w256d128:-:$A --groups 256 --wide-degree 128" \
  "w256d512:-:$A --groups 256 --wide-degree 512" "w256d2k:-:$A --groups 256 --wide-degree 2048" \
  "w128d32b:-:$A --groups 128" "w256d32b:-:$A --groups 256" || exit $?
