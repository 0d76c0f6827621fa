#!/bin/bash
# Sweep the list schedule's task costs (ARSLAM_SIM_COST = POTRF base, per folded column, fused TRSM,
# TRSM, update base, per column, INV; microseconds) on the cfg3 bench: k_factor_dag us per setting.
set -o pipefail
mkdir -p gpurun_out
for c in "$@"; do
  ARSLAM_SIM_COST=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-incremental --no-localize --steps 8 --warmup 2 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sw.json')); print(sys.argv[1], 'dom us', round(d['roofline']['avg_launch_us'],1), 'LM it/s', round(d['value'],1))" "$c"
done
