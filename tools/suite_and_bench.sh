#!/bin/bash
# tools/suite_and_bench.sh <tag>: the whole GPU suite, then one bench line (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh suite_$1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$1.json 2> gpurun_out/bench_$1.err || { tail -30 gpurun_out/bench_$1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$1.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['phase_ms_per_solve'], d['incremental_cfg2']['wall_s'], d['incremental_cfg2']['minimizer_ms_per_solve'], d['localize_cfg5']['value'], d['setup_time_s'])"
