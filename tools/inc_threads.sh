#!/bin/bash
# the incremental cfg2 flow's setup phases with the host worker threads on and off (debug)
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
for th in 16 1; do
  ARSLAM_HOST_THREADS=$th ARSLAM_SETUP_PROFILE=1 timeout -k 10 300 python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_th$th.json 2> gpurun_out/inc_th$th.err || { tail gpurun_out/inc_th$th.err; exit 1; }
  echo "== threads $th"; python3 -c "import json; d=json.load(open('gpurun_out/inc_th$th.json')); print(round(d['wall_s'],3), 'setup', round(d['setup_ms_per_solve'],3), 'min', round(d['minimizer_ms_per_solve'],3))"
  python3 tools/setup_summary.py gpurun_out/inc_th$th.err | grep -E "^setup|^layout"
done
for th in 16 1; do
  ARSLAM_HOST_THREADS=$th timeout -k 10 300 python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_nt$th.json 2>&1 || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/inc_nt$th.json')); print('no profile, threads $th:', round(d['wall_s'],3), 'setup', round(d['setup_ms_per_solve'],3), 'min', round(d['minimizer_ms_per_solve'],3))"
done
