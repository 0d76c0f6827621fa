#!/bin/bash
# Incremental cfg2 flow under several persistent-executor grid sizes (ARSLAM_DAG_GRID)
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
for gsz in default 256 128 64; do
  if [ $gsz = default ]; then unset ARSLAM_DAG_GRID; else export ARSLAM_DAG_GRID=$gsz; fi
  timeout -k 10 200 python tools/bench_incremental.py cfg2 > gpurun_out/inc_$gsz.json 2> gpurun_out/inc_$gsz.err || { tail gpurun_out/inc_$gsz.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/inc_$gsz.json')); print('$gsz', round(d['wall_s'],3), 's', round(d['setup_ms_per_solve'],3), round(d['minimizer_ms_per_solve'],3), 'ms/solve')"
done
