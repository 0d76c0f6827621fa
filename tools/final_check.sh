#!/bin/bash
# end-of-session check on the box: the -m gpu suite, the default bench line, and the executor grid A/B
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
bash tools/gpu_tests.sh gpu_tests_final || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['setup_time_s'], d['incremental_cfg2']['wall_s'])"
timeout -k 10 600 python -u tools/ab.py cfg3 4 base env:ARSLAM_DAG_GRID=448 2>&1 | tee gpurun_out/ab_grid448.txt | tail -2
