#!/bin/bash
# rocprof kernel stats and the PMC HBM passes of the cfg3 bench (no runtime
# warm-up solve, so the per-kernel averages hold only cfg3's launches)
set -o pipefail
export TMPDIR=/tmp
t=${1:-r04}
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
bash tools/prof_bench.sh $t --steps 10 --warmup 2 > gpurun_out/prof_${t}_summary.txt || exit 1
cp $(find gpurun_out/prof_$t -name "*kernel_stats.csv") gpurun_out/kernel_stats_$t.csv
python3 tools/kstats.py gpurun_out/kernel_stats_$t.csv > gpurun_out/kernel_stats_$t.txt
rm -rf gpurun_out/prof_$t
bash tools/pmc_bench.sh $t --steps 3 --warmup 1 || exit 1
rm -rf gpurun_out/pmc_${t}_FETCH_SIZE gpurun_out/pmc_${t}_WRITE_SIZE
head -4 gpurun_out/kernel_stats_$t.txt
grep -o '"avg_launch_us": [0-9.]*' gpurun_out/prof_$t.log | head -1
python3 -c "import json; d=json.load(open('gpurun_out/pmc_$t.json')); print('dominant', d['dominant'], d['hbm_bytes_per_launch'], d['kernels'][d['dominant']]['launches'])"
