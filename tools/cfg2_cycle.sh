#!/bin/bash
# cfg2 on the box: bench line with phases, one DAG trace (critical path), the incremental flow.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-incremental --no-localize --steps 10 --warmup 2 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -30 gpurun_out/c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c2.json')); print('cfg2 LM it/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3), 'iters', d['lm_iterations_per_solve'], d['phase_ms_per_solve'], 'dom us', round(d['roofline']['avg_launch_us'],1))"
ARSLAM_DAG_TRACE=gpurun_out/dag2.bin ARSLAM_DAG_TRACE_SKIP=3 timeout -k 10 200 python bench.py --config cfg2 --no-cpu-baseline --no-incremental --no-localize --steps 1 --warmup 1 > gpurun_out/tr2.log 2>&1 || { tail gpurun_out/tr2.log; exit 1; }
python tools/dag_critical.py gpurun_out/dag2.bin > gpurun_out/crit2.txt; head -14 gpurun_out/crit2.txt
ARSLAM_SETUP_PROFILE=1 timeout -k 10 200 python tools/bench_incremental.py cfg2 > gpurun_out/inc.log 2> gpurun_out/inc.err || { tail -5 gpurun_out/inc.err; exit 1; }
tail -3 gpurun_out/inc.log
