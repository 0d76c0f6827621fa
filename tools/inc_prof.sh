#!/bin/bash
# rocprofv3 kernel stats (and the gzipped kernel trace) of the incremental cfg2 flow (tools/bench_incremental.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inc -o run --output-format csv -- \
  python3 tools/bench_incremental.py cfg2 > gpurun_out/prof_inc.log 2>&1 || { tail gpurun_out/prof_inc.log; exit 1; }
tail -1 gpurun_out/prof_inc.log
python3 tools/kstats.py $(find gpurun_out/prof_inc -name "*kernel_stats.csv") > gpurun_out/kstats_inc.txt
head -25 gpurun_out/kstats_inc.txt
cp $(find gpurun_out/prof_inc -name "*kernel_stats.csv") gpurun_out/kernel_stats_inc.csv
gzip -c $(find gpurun_out/prof_inc -name "*kernel_trace.csv") > gpurun_out/kernel_trace_inc.csv.gz
rm -rf gpurun_out/prof_inc
