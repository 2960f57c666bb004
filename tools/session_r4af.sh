#!/bin/bash
# Round-4 GPU session af: gamma2 only on skewed graphs — tests, then uniform / RMAT configs.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -m gpu > gpurun_out/pt_af.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt_af.log; [ $rc -eq 0 ] || exit 1
U="python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 5"
for i in 1 2; do
  timeout -k 10 300 $U --trace-out gpurun_out/uaf$i.json > gpurun_out/uaf$i.log 2>&1 || exit $?
  echo "uniform $(grep -o '"ms": [0-9.]*' gpurun_out/uaf$i.log)"
done
bash tools/ab.sh "g1024:-:--steps 10" "g16:-:--groups 16 --steps 10" "r22:-:--scale 22 --groups 64 --steps 20"
