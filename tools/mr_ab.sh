#!/bin/bash
# one-rank RCCL multi-rank path: the current library against var_head, interleaved
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
for r in 1 2 3; do
  for v in base head; do
    if [ $v = base ]; then unset ARSLAM_LIB; else export ARSLAM_LIB=$PWD/ar_slam_amd/var_head.so; fi
    timeout -k 10 200 python3 bench.py --rccl-one-rank --steps 5 --warmup 2 --no-cpu-baseline --no-incremental --no-localize --no-fingerprint > gpurun_out/mr_$v.json 2> gpurun_out/mr_$v.err || { tail gpurun_out/mr_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/mr_$v.json').read().strip().splitlines()[-1]); print('round $r', '$v', round(d['value'],1), d['ms_per_step'])" | tee -a gpurun_out/mr_ab.txt
  done
done
