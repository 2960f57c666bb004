#!/bin/bash
# Round-4 GPU session ad: re-measure the README's older rows on the round-4 code.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run NAME LIMIT cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*' gpurun_out/$name.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
run g16 300 python bench.py --groups 16 --steps 10 --warmup 3
run uni 400 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 5
run dist16 300 python bench.py --algo dist --groups 16 --steps 3 --warmup 1
run sweep2 300 python bench.py --algo sweep --groups 2 --steps 1 --warmup 0 --verify 0
run r30 900 python bench.py --scale 30 --groups 256 --steps 2 --warmup 1 --verify 0
