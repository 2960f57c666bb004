#!/bin/bash
# GPU-box session runner: each step has its own time limit; stop at the first fault/abort/timeout
# (exit status > 1); plain test failures (status 1) are recorded and the session continues.
#   tools/gpu_session.sh pytest bench26 prof26 ...
# Tuning experiments go through MSBFS_TUNE="key=value,..." (validated, echoed on stderr).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name (limit ${limit}s): $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
  # a GPU fault inside a Python process surfaces as an exception (status 1): stop there too
  if grep -qE "illegal memory access|Memory access fault|hipErrorLaunchFailure|HSA_STATUS_ERROR" \
      "gpurun_out/$name.log"; then echo "stopping: GPU fault in $name"; exit 3; fi
  return 0
}
prof() {  # prof NAME LIMIT args...: kernel trace + stats of one command, summary in NAME.md
  local name=$1 limit=$2; shift 2
  export TMPDIR=/tmp; rm -rf "gpurun_out/$name"
  step "$name" "$limit" rocprofv3 --kernel-trace --stats -T --output-format csv \
    -d "gpurun_out/$name" -o run -- "$@" &&
  python tools/prof_summary.py "gpurun_out/$name" > "gpurun_out/$name.md" &&
  rm -f "gpurun_out/$name/run_kernel_trace.csv"
}
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 1100 $PT tests -m gpu ;;
    pytest_kernels) step pytest_kernels 900 $PT tests/test_gpu_kernels.py -m gpu ;;
    pytest_rest) step pytest_rest 900 $PT tests -m gpu --deselect tests/test_gpu_kernels.py ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    bench26) step bench26 300 python bench.py --steps 20 --warmup 5 ;;
    bench2r) step bench2r 600 python bench.py --gpus 2 --backend gloo --scale 22 --steps 2 --warmup 1 ;;
    trace26) MSBFS_TRACE=1 step trace26 300 python bench.py --steps 2 --warmup 1 ;;
    trace128) MSBFS_TRACE=1 step trace128 300 python bench.py --steps 2 --warmup 1 --groups 128 ;;
    prof26) prof prof26 600 python bench.py --steps 1 --warmup 0 --verify 0 ;;
    prof128) prof prof128 600 python bench.py --groups 128 --steps 1 --warmup 0 --verify 0 ;;
    prof256) prof prof256 600 python bench.py --groups 256 --steps 1 --warmup 0 --verify 0 ;;
    prof512) prof prof512 600 python bench.py --groups 512 --steps 1 --warmup 0 --verify 0 ;;
    prof30) prof prof30 900 python bench.py --scale 30 --groups 32 --steps 1 --warmup 1 --verify 0 ;;
    prof22) prof prof22 300 python bench.py --scale 22 --groups 64 --steps 3 --warmup 1 --verify 0 ;;
    rmat22) step rmat22 300 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1 --verify 16 ;;
    rmat30) MSBFS_TRACE=1 step rmat30 1000 python bench.py --scale 30 --groups 256 --steps 1 --warmup 0 ;;
    road) step road 900 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64 --steps 1 --verify 2 ;;
    road16) step road16 900 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 16 --steps 1 ;;
    profroad) prof profroad 900 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64 --steps 1 ;;
    uniform) step uniform 600 python tools/bench_graph.py --graph uniform:16000000:128000000 --groups 1024 --steps 3 ;;
    exitrt)  # teardown under the runtime tracer, least to most state (stops at the first crash)
      export TMPDIR=/tmp
      for m in ${EXIT_MODES:-torch tsolve tbig bench}; do
        if [ $m = bench ]; then cmd="python bench.py --steps 2 --warmup 1 --verify 0"
        else cmd="python tools/exit_check.py $m"; fi
        step exitrt_$m 300 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/exrt_$m \
          -o run -- $cmd
      done ;;
    hybsim) step hybsim 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 ;;
    hybsim8) step hybsim8 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin ;;
    profhyb8) prof profhyb 900 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin ;;
    profhc)  # kernel timelines of phase C of ranks 0 and 1 (8 emulated ranks)
      export TMPDIR=/tmp; rm -rf gpurun_out/profhc
      step profhc 900 rocprofv3 --kernel-trace --stats -T --output-format csv \
        -d gpurun_out/profhc -o run -- python tools/hybrid_sim.py --scale 26 --ranks 8 \
        --no-roundrobin --chunks 4 &&
      for k in 8 7; do PROF_START=k_hybrid_setup PROF_NTH=$k python tools/prof_summary.py \
        gpurun_out/profhc > "gpurun_out/profhc_r$((8 - k)).md"; done &&
      PROF_START=k_init PROF_NTH=8 python tools/prof_summary.py gpurun_out/profhc \
        > gpurun_out/profhc_a0.md &&
      rm -f gpurun_out/profhc/run_kernel_trace.csv ;;
    pmchbm) export TMPDIR=/tmp; R="${PMC_RE:-k_bu|k_push|k_pfx|k_build}"; rm -rf gpurun_out/pmch1 gpurun_out/pmch2 gpurun_out/pmch3
         step pmch1 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch1 -o run -- python bench.py --steps 1 --warmup 0 --verify 0 &&
         step pmch2 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch2 -o run -- python bench.py --steps 1 --warmup 0 --verify 0 &&
         step pmch3 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TA_BUSY_avr --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch3 -o run -- python bench.py --steps 1 --warmup 0 --verify 0 &&
         for d in pmch1 pmch2 pmch3; do python tools/prof_summary.py gpurun_out/$d > gpurun_out/$d.md; done ;;
    pmcregex) # PMC_RE=<kernel regex>: three counter passes of one timed RMAT-26 step
         export TMPDIR=/tmp; R="${PMC_RE:-k_pfx_tiles}"; rm -rf gpurun_out/pmcr1 gpurun_out/pmcr2 gpurun_out/pmcr3
         B="${PMC_B:-python bench.py --steps 1 --warmup 0 --verify 0}"
         step pmcr1 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcr1 -o run -- $B &&
         step pmcr2 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcr2 -o run -- $B &&
         step pmcr3 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcr3 -o run -- $B &&
         for d in pmcr1 pmcr2 pmcr3; do python tools/prof_summary.py gpurun_out/$d > gpurun_out/$d.md; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
