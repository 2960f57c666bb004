#!/bin/bash
# Round-4 GPU session ae: uniform random graph (n = 16M, m = 128M, 1024 groups) 34 ms now vs 27.2
# in round 2 — per-level records with the default, gamma2 = gamma, a forced second push level and
# relabelled ids.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run NAME ENV cmd...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 "$@" --trace-out gpurun_out/$name.json > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"ms": [0-9.]*' gpurun_out/$name.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
  python - "gpurun_out/$name.json" <<'PY'
import json, sys
t = json.load(open(sys.argv[1]))
print("   ", " ".join(f"{r['dir']}{r['ms']:.2f}" for r in t))
PY
}
U="python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 5"
run u0 MSBFS_X=0 $U
run ug MSBFS_TUNE=gamma2=-1 $U
run ut MSBFS_TUNE=dirs=TT $U
run ur MSBFS_X=0 $U --relabel 1
run utr MSBFS_TUNE=dirs=TT $U --relabel 1
