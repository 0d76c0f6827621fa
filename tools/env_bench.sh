#!/bin/bash
# A/B of plan/executor environment settings on the cfg3 bench, interleaved.
# usage (on the box): bash tools/env_bench.sh "ENV=1 ENV2=2" "ENV=3" ...   ("" = default)
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 120 python bench.py --no-cpu-baseline --no-incremental --steps 10 --warmup 2 > gpurun_out/eb_$i.json 2> gpurun_out/eb_$i.err || { tail -5 gpurun_out/eb_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/eb_$i.json')); print('[$v]', round(d['value'],1), 'it/s', round(d['ms_per_step'],3), 'ms', round(d['roofline']['avg_launch_us'],1), 'us factor')"
  done
done
