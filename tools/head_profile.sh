#!/bin/bash
# the default bench line and the rocprofv3 kernel stats at HEAD (round 4 close)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
t=${1:-r04c}
timeout -k 10 300 python bench.py > gpurun_out/bench_$t.json 2> gpurun_out/bench_$t.err || { tail -30 gpurun_out/bench_$t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$t.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['setup_time_s'], d['incremental_cfg2']['wall_s'])"
bash tools/prof_bench.sh $t --steps 10 --warmup 2 > gpurun_out/prof_${t}_summary.txt || exit 1
cp $(find gpurun_out/prof_$t -name "*kernel_stats.csv") gpurun_out/kernel_stats_$t.csv
python3 tools/kstats.py gpurun_out/kernel_stats_$t.csv > gpurun_out/kernel_stats_$t.txt
rm -rf gpurun_out/prof_$t
head -6 gpurun_out/kernel_stats_$t.txt
