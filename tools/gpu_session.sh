#!/bin/bash
# GPU-box session runner: each step has its own time limit; stop at the first fault/abort/timeout
# (exit status > 1); plain test failures (status 1) are recorded and the session continues.
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
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    smoke) step smoke 300 python __graft_entry__.py smoke ;;
    bench20) step bench20 300 python bench.py --scale 20 --steps 3 --warmup 1 --verify 32 ;;
    bench22) step bench22 300 python bench.py --scale 22 --steps 3 --warmup 1 --verify 16 ;;
    bench26) step bench26 900 python bench.py --steps 3 --warmup 1 ;;
    trace26) MSBFS_TRACE=1 step trace26 600 python bench.py --steps 2 --warmup 0 ;;
    prof26) export TMPDIR=/tmp; step prof26 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof26 -o run -- python bench.py --steps 1 --warmup 0 ;;
    sweep26) step sweep26 900 python bench.py --algo sweep --groups 4 --steps 1 --warmup 0 ;;
    dist26) step dist26 900 python bench.py --algo dist --groups 16 --steps 1 --warmup 0 ;;
    verify26) step verify26 900 python bench.py --steps 1 --warmup 0 --verify 64 ;;
    filt0) MSBFS_FILTER_FRAC=0 MSBFS_TRACE=1 step filt0 600 python bench.py --steps 2 --warmup 0 ;;
    filt2) MSBFS_FILTER_FRAC=2 MSBFS_TRACE=1 step filt2 600 python bench.py --steps 2 --warmup 0 ;;
    unroll8) MSBFS_UNROLL=8 MSBFS_TRACE=1 step unroll8 600 python bench.py --steps 2 --warmup 0 ;;
    words8) MSBFS_TRACE=1 step words8 600 python bench.py --steps 2 --warmup 0 --max-words 8 ;;
    wide32) MSBFS_TRACE=1 step wide32 600 python bench.py --steps 2 --warmup 0 --wide-degree 32 ;;
    wide256) MSBFS_TRACE=1 step wide256 600 python bench.py --steps 2 --warmup 0 --wide-degree 256 ;;
    wl128) MSBFS_WIDE_LATER=128 MSBFS_TRACE=1 step wl128 600 python bench.py --steps 2 --warmup 0 ;;
    wl1024) MSBFS_WIDE_LATER=1024 MSBFS_TRACE=1 step wl1024 600 python bench.py --steps 2 --warmup 0 ;;
    pmc) export TMPDIR=/tmp
         step pmclist 120 rocprofv3 -L
         step pmc1 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_bu|k_count" --output-format csv -d gpurun_out/pmc1 -o run -- python bench.py --steps 1 --warmup 0
         step pmc2 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_bu|k_count" --output-format csv -d gpurun_out/pmc2 -o run -- python bench.py --steps 1 --warmup 0
         step pmc3 600 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --kernel-include-regex "k_bu|k_count" --output-format csv -d gpurun_out/pmc3 -o run -- python bench.py --steps 1 --warmup 0
         ;;
    g512) MSBFS_TRACE=1 step g512 600 python bench.py --steps 3 --warmup 1 --groups 512 ;;
    g256) MSBFS_TRACE=1 step g256 600 python bench.py --steps 3 --warmup 1 --groups 256 ;;
    g128) MSBFS_TRACE=1 step g128 600 python bench.py --steps 3 --warmup 1 --groups 128 ;;
    g64) MSBFS_TRACE=1 step g64 600 python bench.py --steps 3 --warmup 1 --groups 64 ;;
    g128f0) MSBFS_FILTER_FRAC=0 MSBFS_TRACE=1 step g128f0 600 python bench.py --steps 3 --warmup 1 --groups 128 ;;
    prof128) export TMPDIR=/tmp; rm -rf gpurun_out/prof128; step prof128 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof128 -o run -- python bench.py --steps 1 --warmup 0 --groups 128 ;;
    pmc128) export TMPDIR=/tmp
         step pmc4 600 rocprofv3 --pmc TCC_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex "k_bu" --output-format csv -d gpurun_out/pmc4 -o run -- python bench.py --steps 1 --warmup 0 --groups 128
         step pmc5 600 rocprofv3 --pmc TA_BUSY_avr TCC_BUSY_avr GRBM_GUI_ACTIVE TA_ADDR_STALLED_BY_TC_CYCLES_sum --kernel-include-regex "k_bu" --output-format csv -d gpurun_out/pmc5 -o run -- python bench.py --steps 1 --warmup 0 --groups 128
         ;;
    hub0) MSBFS_HUB_MB=0 MSBFS_TRACE=1 step hub0 600 python bench.py --steps 3 --warmup 1 ;;
    hub64) MSBFS_HUB_MB=64 MSBFS_TRACE=1 step hub64 600 python bench.py --steps 3 --warmup 1 ;;
    hub128g) MSBFS_HUB_MB=64 MSBFS_TRACE=1 step hub128g 600 python bench.py --steps 3 --warmup 1 --groups 128 ;;
    hub4g) MSBFS_HUB_MB=4 MSBFS_TRACE=1 step hub4g 600 python bench.py --steps 3 --warmup 1 --groups 128 ;;
    mr2) step mr2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --scale 22 --steps 2 --warmup 1 --backend gloo ;;
    mr1) step mr1 600 python bench.py --scale 22 --steps 2 --warmup 1 ;;
    road) step road_bp 600 python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 256 --verify 4
          step road_dist 600 python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 8 --algo dist --steps 1 ;;
    profroad) export TMPDIR=/tmp; step profroad 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profroad -o run -- python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 256 --steps 1 ;;
    dirs128) MSBFS_DIRS=TTBBBBBB MSBFS_TRACE=1 step d128_ttb 600 python bench.py --steps 3 --warmup 1 --groups 128
             MSBFS_DIRS=TTTBBBBB MSBFS_TRACE=1 step d128_tttb 600 python bench.py --steps 3 --warmup 1 --groups 128
             MSBFS_TRACE=1 step d128_auto 600 python bench.py --steps 3 --warmup 1 --groups 128
             MSBFS_DIRS=TTBBBBBB MSBFS_TRACE=1 step d1024_ttb 600 python bench.py --steps 3 --warmup 1 ;;
    hybtest) step hybtest 900 python -m pytest tests/test_hybrid.py -m gpu -x -q ;;
    hybsim) step hybsim 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 ;;
    hybsim22) step hybsim22 600 python tools/hybrid_sim.py --scale 22 --ranks 2 8 ;;
    profhyb) export TMPDIR=/tmp; rm -rf gpurun_out/profhyb; step profhyb 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profhyb -o run -- python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin ;;
    hyb2) step hyb2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --scale 22 --steps 2 --warmup 1 --backend gloo --dist hybrid ;;
    road2) step road_td 600 python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 256 --force-dir 1
           step road_a2 600 python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 256 --alpha 2
           step road_1024 600 python tools/bench_graph.py --graph grid:2048:2048:0.7 --groups 1024 --force-dir 1
           step rmat_a4 600 python tools/bench_graph.py --graph rmat:24:16 --groups 1024 --alpha 4 --relabel 1
           step rmat_a14 600 python tools/bench_graph.py --graph rmat:24:16 --groups 1024 --relabel 1 ;;
    rmat22) step rmat22 300 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1 --verify 16 ;;
    usaroad) step usaroad 900 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64 --steps 1 ;;
    hyb8trace) MSBFS_TRACE=1 step hyb8trace 600 python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin ;;
    hyb4trace) MSBFS_TRACE=1 step hyb4trace 600 python tools/hybrid_sim.py --scale 26 --ranks 4 --no-roundrobin ;;
    pmcnarrow) export TMPDIR=/tmp
         step pmcn1 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_bu_narrow" --output-format csv -d gpurun_out/pmcn1 -o run -- python bench.py --steps 1 --warmup 0 --groups 128
         step pmcn2 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex "k_bu_narrow" --output-format csv -d gpurun_out/pmcn2 -o run -- python bench.py --steps 1 --warmup 0 --groups 128
         step pmcn3 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "k_bu_narrow" --output-format csv -d gpurun_out/pmcn3 -o run -- python bench.py --steps 1 --warmup 0 --groups 128
         ;;
    t26) MSBFS_TRACE=1 step t26 300 python bench.py --steps 2 --warmup 1 ;;
    pmcbu) export TMPDIR=/tmp; R="k_bu_chunks|k_bu_narrow"
         step pmcb1 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcb1 -o run -- python bench.py --steps 1 --warmup 0
         step pmcb2 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcb2 -o run -- python bench.py --steps 1 --warmup 0
         step pmcb3 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcb3 -o run -- python bench.py --steps 1 --warmup 0
         ;;
    t26v) MSBFS_TRACE=1 step t26v 300 python bench.py --steps 2 --warmup 1 --verify 64 ;;
    c26) for d in 1 4; do MSBFS_CODE_DEG=$d MSBFS_TRACE=1 step c26_$d 300 python bench.py --steps 2 --warmup 1; done ;;
    hubbig) for b in 1 2 3; do MSBFS_HUBBIG=$b MSBFS_TRACE=1 step hubbig$b 300 python bench.py --steps 2 --warmup 1; done
            MSBFS_HUBBIG=3 MSBFS_TRACE=1 step hubbig3g128 300 python bench.py --steps 2 --warmup 1 --groups 128 ;;
    pfx2) MSBFS_PFX=2 MSBFS_TRACE=1 step pfx2_26 300 python bench.py --steps 2 --warmup 1 --verify 16
          MSBFS_PFX=2 MSBFS_TRACE=1 step pfx2_128 300 python bench.py --steps 2 --warmup 1 --groups 128 ;;
    pfxh) for h in 65536 131072 262144; do MSBFS_PFX=2 MSBFS_PFX_H=$h MSBFS_TRACE=1 step pfxh_$h 300 python bench.py --steps 2 --warmup 1
          MSBFS_PFX=2 MSBFS_PFX_H=$h MSBFS_TRACE=1 step pfxh128_$h 300 python bench.py --steps 2 --warmup 1 --groups 128; done ;;
    narrowc) for c in 1 2; do MSBFS_NARROW_C=$c MSBFS_TRACE=1 step nc$c 300 python bench.py --steps 2 --warmup 1 --verify 16
            MSBFS_NARROW_C=$c MSBFS_TRACE=1 step nc128_$c 300 python bench.py --steps 2 --warmup 1 --groups 128; done ;;
    hyb2trace) MSBFS_TRACE=1 step hyb2trace 600 python tools/hybrid_sim.py --scale 26 --ranks 2 --no-roundrobin ;;
    hybsimall) step hybsimall 900 python tools/hybrid_sim.py --scale 26 --ranks 2 4 8 ;;
    hybpfx) for x in 2 0 1; do MSBFS_PFX=$x step hybpfx_$x 600 python tools/hybrid_sim.py --scale 26 --ranks 4 8 --no-roundrobin; done ;;
    regen) step regen 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "regeneration or relabelled" ;;
    rmat30) MSBFS_TRACE=1 step rmat30 1000 python bench.py --scale 30 --groups 256 --steps 1 --warmup 0 ;;
    prof30) export TMPDIR=/tmp; rm -rf gpurun_out/prof30; step prof30 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof30 -o run -- python bench.py --scale 30 --groups 256 --steps 1 --warmup 0 &&
            python tools/prof_summary.py gpurun_out/prof30 > gpurun_out/prof30.md && rm -f gpurun_out/prof30/run_kernel_trace.csv ;;
    r30coop) for x in -1 0; do MSBFS_COOP=$x MSBFS_TRACE=1 step r30coop_$x 600 python bench.py --scale 30 --groups 256 --steps 1 --warmup 0; done &&
             MSBFS_DIRS=TBBBBBBBBBBBBBBBBBBB MSBFS_TRACE=1 step r30tb 600 python bench.py --scale 30 --groups 256 --steps 1 --warmup 0 ;;
    alpha) for a in 14 32 64; do
             step al22_$a 300 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1 --alpha $a &&
             step al26g16_$a 300 python bench.py --groups 16 --steps 3 --warmup 1 --alpha $a &&
             step al26g128_$a 300 python bench.py --groups 128 --steps 3 --warmup 1 --alpha $a &&
             step al26_$a 300 python bench.py --steps 3 --warmup 1 --alpha $a &&
             step al30_$a 600 python bench.py --scale 30 --groups 256 --steps 1 --warmup 0 --alpha $a &&
             step alroad_$a 600 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64 --steps 1 --alpha $a || exit 1; done ;;
    dirchk) step dc22 300 python bench.py --scale 22 --groups 64 --steps 5 --warmup 1 --verify 16 &&
            step dc26g16 300 python bench.py --groups 16 --steps 3 --warmup 1 --verify 4 &&
            step dc26g128 300 python bench.py --groups 128 --steps 3 --warmup 1 &&
            step dc26 300 python bench.py --steps 3 --warmup 1 &&
            step dc30 600 python bench.py --scale 30 --groups 256 --steps 2 --warmup 1 &&
            step dcroad 600 python tools/bench_graph.py --graph grid:4896:4896:0.6 --groups 64 --steps 1 ;;
    profhyb8) export TMPDIR=/tmp; rm -rf gpurun_out/profhyb; step profhyb8 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/profhyb -o run -- python tools/hybrid_sim.py --scale 26 --ranks 8 --no-roundrobin &&
              python tools/prof_summary.py gpurun_out/profhyb > gpurun_out/profhyb.md && rm -f gpurun_out/profhyb/run_kernel_trace.csv ;;
    lazy) for x in 1 0; do MSBFS_LAZY=$x step lazy_$x 600 python tools/hybrid_sim.py --scale 26 --ranks 4 8 --no-roundrobin || exit 1; done ;;
    aq) for x in 4096 1024 4096 1024; do MSBFS_AQ=$x step aq_$x 300 python bench.py --steps 3 --warmup 1 || exit 1; grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/aq_$x.log; done ;;
    ab) for x in a b; do step ab26_$x 300 python bench.py --steps 5 --warmup 2 || exit 1; grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/ab26_$x.log; done
        step ab128 300 python bench.py --steps 5 --warmup 2 --groups 128 || exit 1; grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/ab128.log ;;
    knobs128) for kv in NONE=0 MSBFS_NARROW_C=0 MSBFS_NARROW_C=1 MSBFS_WIDE_LATER=128 MSBFS_WIDE_LATER=1024 MSBFS_FILTER_FRAC=0 MSBFS_FILTER_FRAC=2 MSBFS_COOP=1 MSBFS_GAMMA=0; do
          n=${kv//=/_}; env "$kv" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --groups 128 > gpurun_out/k128_$n.log 2>&1 || exit 1
          echo "$kv $(grep -o '"ms_per_step": [0-9.]*\|"level_ms": [^]]*' gpurun_out/k128_$n.log | tr '\n' ' ')"; done ;;
    pmclds) export TMPDIR=/tmp; rm -rf gpurun_out/pmcb3
         step pmcb3 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM --kernel-include-regex "k_bu_chunks|k_bu_narrow" --output-format csv -d gpurun_out/pmcb3 -o run -- python bench.py --steps 1 --warmup 0 ;;
    pmchbm) export TMPDIR=/tmp; R="k_bu|k_push|k_td|k_build|k_level"; rm -rf gpurun_out/pmch1 gpurun_out/pmch2 gpurun_out/pmch3
         step pmch1 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch1 -o run -- python bench.py --steps 1 --warmup 0 &&
         step pmch2 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch2 -o run -- python bench.py --steps 1 --warmup 0 &&
         step pmch3 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TA_BUSY_avr --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmch3 -o run -- python bench.py --steps 1 --warmup 0 &&
         for d in pmch1 pmch2 pmch3; do python tools/prof_summary.py gpurun_out/$d > gpurun_out/$d.md; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
