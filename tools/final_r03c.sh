#!/bin/bash
# Round-3 (third part) closing set on the box: the full GPU suite, the default
# bench line, rocprofv3 kernel stats (cfg3 and the incremental cfg2 flow), PMC
# HBM bytes and SQ counters; bulky rocprof directories removed.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
touch ar_slam_amd/*.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r03c.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_r03c.txt; exit 1; }
tail -1 gpurun_out/gpu_tests_r03c.txt
bash tools/profile_r03c.sh || exit 1
bash tools/inc_prof.sh || exit 1
ARSLAM_SETUP_PROFILE=1 timeout -k 10 200 python tools/bench_incremental.py cfg2 > gpurun_out/inc_setup.json 2> gpurun_out/inc_setup.err || { tail gpurun_out/inc_setup.err; exit 1; }
python3 tools/setup_prof.py gpurun_out/inc_setup.err | tee gpurun_out/inc_setup_phases.txt
