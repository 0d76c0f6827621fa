#!/bin/bash
# executor grid size on the small configs and the incremental flow (debug)
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
timeout -k 10 400 python -u tools/ab.py cfg2 3 base env:ARSLAM_DAG_GRID=256 env:ARSLAM_DAG_GRID=128 env:ARSLAM_DAG_GRID=64 2>&1 | tee gpurun_out/ab_grid_cfg2.txt | grep median
for gsz in 448 128; do
  ARSLAM_DAG_GRID=$gsz timeout -k 10 300 python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_g$gsz.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/inc_g$gsz.json')); print('grid $gsz:', round(d['wall_s'],3), 'setup', round(d['setup_ms_per_solve'],3), 'min', round(d['minimizer_ms_per_solve'],3))"
done
