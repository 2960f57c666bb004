set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -rf gpurun_out/prof26 gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC
R="k_bu_chunks|k_bu_narrow|k_push_tail|k_bu_wide_finalize"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof26 -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/prof26.log 2>&1
python tools/prof_summary.py gpurun_out/prof26 > gpurun_out/prof26.md
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcA -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/pmcA.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcB -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/pmcB.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TD_BUSY_avr TCC_EA0_RDREQ_sum WRITE_SIZE --kernel-include-regex "$R" --output-format csv -d gpurun_out/pmcC -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/pmcC.log 2>&1
for d in pmcA pmcB pmcC; do python tools/prof_summary.py gpurun_out/$d > gpurun_out/$d.md; done
rm -f gpurun_out/prof26/run_kernel_trace.csv
