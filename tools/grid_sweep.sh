#!/bin/bash
# Persistent-executor grid sweep on the box: cfg3 bench line per ARSLAM_DAG_GRID value.
# usage: bash tools/grid_sweep.sh 256 384 512
mkdir -p gpurun_out
for g in "$@"; do
  ARSLAM_DAG_GRID=$g timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/grid_$g.json 2> gpurun_out/grid_$g.err || { tail -5 gpurun_out/grid_$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/grid_$g.json')); print('grid $g', round(d['value'],1), 'LM it/s', d['phase_ms_per_solve']['cholesky'], d['phase_ms_per_solve']['solve'])"
done
