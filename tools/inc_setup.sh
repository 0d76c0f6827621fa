#!/bin/bash
# the incremental cfg2 flow with the host setup phases (ARSLAM_SETUP_PROFILE) summarised (debug)
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
ARSLAM_SETUP_PROFILE=1 timeout -k 10 300 python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_setup.json 2> gpurun_out/inc_setup.err || { tail gpurun_out/inc_setup.err; exit 1; }
cat gpurun_out/inc_setup.json
python3 tools/setup_summary.py gpurun_out/inc_setup.err
