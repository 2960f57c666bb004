#!/bin/bash
# Kernel-level A/B on the GPU box: for each "<label>:<env>:<bench args>", one rocprofv3 kernel
# trace of bench.py, then per-kernel time of the LAST solver run (tools/prof_summary.py timeline).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r label envs args <<< "$spec"
  envcmd=()
  if [ "$envs" != "-" ]; then IFS=, read -ra envcmd <<< "$envs"; fi
  d=gpurun_out/k_$label
  rm -rf "$d"
  env "${envcmd[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- python bench.py $args > "$d.log" 2>&1
  rc=$?
  echo "== $label rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $d.log)"
  # (rc 3 = bench's self-check failed: expected for timing-only variants that drop correctness)
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -5 "$d.log"; exit $rc; fi
  python tools/prof_summary.py "$d" | sed -n '/Timeline/,$p' | grep -v "^$" | awk -F'|' 'NR>4 && $7+0 > 0.05 {printf "%s %s|", $3, $7} END {print ""}'
  rm -f "$d/run_kernel_trace.csv"
done
