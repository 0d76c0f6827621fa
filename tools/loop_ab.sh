#!/bin/bash
# A/B of the LM loop on the box: cfg3 and cfg2 bench lines, host loop vs device loop
# (with and without the dominant kernel's timing events), interleaved.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in cfg3 cfg2; do
    for v in host dev dev_nograph; do
      case $v in
        host) f=""; unset ARSLAM_LOOP_NOGRAPH;;
        dev) f="--device-loop"; unset ARSLAM_LOOP_NOGRAPH;;
        dev_nograph) f="--device-loop"; export ARSLAM_LOOP_NOGRAPH=1;;
      esac
      timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --no-incremental --no-localize --steps 10 --warmup 2 $f > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
      python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); r=d.get('roofline') or {}; print(sys.argv[1], sys.argv[2], 'LM it/s', round(d['value'],1), 'ms', round(d['ms_per_step'],3), 'loop', d.get('lm_loop'), 'dom us', round(r.get('avg_launch_us') or 0,1))" $cfg $v
    done
  done
done
