#!/bin/bash
# Round-4 profile set on the box: the whole GPU suite, the default bench line,
# rocprofv3 kernel stats (cfg3 and the incremental cfg2 flow), PMC HBM bytes
# (FETCH_SIZE and WRITE_SIZE passes) and SQ counters; bulky rocprof
# directories removed after their summaries.  usage: bash tools/profile_r04.sh <tag>
set -o pipefail
export TMPDIR=/tmp
t=${1:-r04b}
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
bash tools/gpu_tests.sh gpu_tests_$t || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_$t.json 2> gpurun_out/bench_$t.err || { tail -30 gpurun_out/bench_$t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$t.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['setup_time_s'], d['incremental_cfg2']['wall_s'], d['localize_cfg5']['value'])"
bash tools/prof_bench.sh $t --steps 10 --warmup 2 > gpurun_out/prof_${t}_summary.txt || exit 1
cp $(find gpurun_out/prof_$t -name "*kernel_stats.csv") gpurun_out/kernel_stats_$t.csv
python3 tools/kstats.py gpurun_out/kernel_stats_$t.csv > gpurun_out/kernel_stats_$t.txt
rm -rf gpurun_out/prof_$t
bash tools/inc_prof.sh > /dev/null || exit 1
bash tools/pmc_bench.sh $t --steps 3 --warmup 1 || exit 1
rm -rf gpurun_out/pmc_${t}_FETCH_SIZE gpurun_out/pmc_${t}_WRITE_SIZE
cat gpurun_out/pmc_$t.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('dominant', d['dominant'], d['hbm_bytes_per_launch'])"
bash tools/pmc_sq.sh occ "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM" > gpurun_out/pmc_sq_$t.txt || exit 1
rm -rf gpurun_out/pmcsq_occ
cat gpurun_out/pmc_sq_$t.txt
bash tools/inc_ab.sh | tee gpurun_out/inc_ab_$t.txt
