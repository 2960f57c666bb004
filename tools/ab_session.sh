#!/bin/bash
# One GPU session of A/B comparisons between the in-tree build and abl/prev (the last commit):
# bench.py configurations, each "new" then "prev" (tools/ab.sh).
set -u
P=abl/prev/libmsbfs.so
for cfg in "$@"; do
  case $cfg in
    r26) A="--steps 20 --warmup 5" ;;
    r26g128) A="--groups 128 --steps 10 --warmup 3" ;;
    r26g16) A="--groups 16 --steps 10 --warmup 3" ;;
    r30g32) A="--scale 30 --groups 32 --steps 2 --warmup 1 --verify 2" ;;
    *) echo "unknown config $cfg"; exit 2 ;;
  esac
  tools/ab.sh "${cfg}_new:-:$A" "${cfg}_prev:MSBFS_LIB=$P:$A" || exit $?
done
