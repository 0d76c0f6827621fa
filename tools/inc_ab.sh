#!/bin/bash
# the incremental cfg2 flow: the host LM loop and the device-resident loop, alternating (debug A/B)
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
for r in 1 2; do
  for dl in 0 1; do
    ARSLAM_DEVICE_LOOP=$dl timeout -k 10 300 python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_dl$dl.json 2>&1 || { tail gpurun_out/inc_dl$dl.json; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/inc_dl$dl.json')); print('device_loop=$dl', round(d['wall_s'],3), 'setup', round(d['setup_ms_per_solve'],3), 'min', round(d['minimizer_ms_per_solve'],3), 'other', round(d['other_ms_per_solve'],3))"
  done
done
