#!/bin/bash
# Full GPU round trip on the box: gpu tests, default bench line, rocprof kernel
# stats, PMC HBM bytes.  Usage: bash tools/round_cycle.sh <tag>
set -o pipefail
tag=${1:-cycle}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
timeout -k 10 240 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -30 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
bash tools/prof_bench.sh $tag --steps 10 --warmup 2 || exit 1
bash tools/pmc_bench.sh $tag --steps 3 --warmup 1 || exit 1
cat gpurun_out/pmc_$tag.json
