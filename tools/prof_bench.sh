#!/bin/bash
# usage (on the GPU box): tools/prof_bench.sh <tag> [bench args...]
# rocprofv3 kernel trace + stats of one bench run; output under gpurun_out/prof_<tag>/
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-incremental --no-runtime-warmup "$@" > gpurun_out/prof_$tag.log 2>&1
rc=$?
tail -1 gpurun_out/prof_$tag.log
python3 tools/kstats.py $(find gpurun_out/prof_$tag -name "*kernel_stats.csv") | head -25
exit $rc
