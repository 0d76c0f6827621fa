#!/bin/bash
# Round-3 (third part) profile set on the box: the default bench line, rocprofv3
# kernel stats, PMC HBM bytes and SQ instruction counters; bulky rocprof
# directories removed after their summaries (gpurun copies back <= 64 MiB).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
touch ar_slam_amd/*.so
timeout -k 10 300 python bench.py > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || { tail -30 gpurun_out/bench_r03c.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03c.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['incremental_cfg2']['wall_s'], d['localize_cfg5']['value'])"
bash tools/prof_bench.sh r03c --steps 10 --warmup 2 > gpurun_out/prof_r03c_summary.txt || exit 1
cp $(find gpurun_out/prof_r03c -name "*kernel_stats.csv") gpurun_out/kernel_stats_r03c.csv
python3 tools/kstats.py gpurun_out/kernel_stats_r03c.csv > gpurun_out/kernel_stats_r03c.txt
rm -rf gpurun_out/prof_r03c
bash tools/pmc_bench.sh r03c --steps 3 --warmup 1 || exit 1
rm -rf gpurun_out/pmc_r03c_FETCH_SIZE gpurun_out/pmc_r03c_WRITE_SIZE
cat gpurun_out/pmc_r03c.json
bash tools/pmc_sq.sh occ "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM" > gpurun_out/pmc_sq_r03c.txt || exit 1
rm -rf gpurun_out/pmcsq_occ
cat gpurun_out/pmc_sq_r03c.txt
