#!/bin/bash
# A/B the default library against variant builds (ar_slam_amd/var_<name>.so,
# built here with ARSLAM_LIB/ARSLAM_EXTRA_FLAGS): cfg3 bench, interleaved.
# usage (on the box): bash tools/variant_bench.sh name1 name2 ...
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then lib=ar_slam_amd/libarslam_lm.so; else lib=ar_slam_amd/var_$v.so; fi
    ARSLAM_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-incremental --steps 10 --warmup 2 > gpurun_out/vb_$v.json 2> gpurun_out/vb_$v.err || { tail -5 gpurun_out/vb_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/vb_$v.json')); print('$v', round(d['value'],1), 'it/s', round(d['ms_per_step'],3), 'ms', round(d['roofline']['avg_launch_us'],1), 'us factor', {k: round(v,3) for k,v in d['phase_ms_per_solve'].items()})"
  done
done
