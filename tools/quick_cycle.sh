#!/bin/bash
# Quick GPU check on the box: gpu tests (optional filter), cfg3 bench line, DAG critical path.
# usage: bash tools/quick_cycle.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
if [ -n "$1" ]; then K=(-k "$1"); else K=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > gpurun_out/qt.log 2>&1 || { tail -40 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/qb.json 2> gpurun_out/qb.err || { tail -30 gpurun_out/qb.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/qb.json')); print('LM it/s', round(d['value'],1), 'ms', round(d['ms_per_step'],2), 'iters', d['lm_iterations_per_solve'], d['phase_ms_per_solve'], 'dom us', round(d['roofline']['avg_launch_us'],1), 'frac', round(d['roofline']['frac'],4))"
ARSLAM_DAG_TRACE=gpurun_out/dag.bin ARSLAM_DAG_TRACE_SKIP=3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-incremental --steps 1 --warmup 1 > gpurun_out/tr.log 2>&1 || { tail gpurun_out/tr.log; exit 1; }
python tools/dag_critical.py gpurun_out/dag.bin > gpurun_out/crit.txt; head -14 gpurun_out/crit.txt
