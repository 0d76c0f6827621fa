#!/bin/bash
# cfg5 batched-localize A/B on the box (debug): the default library and variants ar_slam_amd/var_<name>.so
# interleaved, ROUNDS times (bench.py --config cfg5).  usage: ROUNDS=3 bash tools/loc_ab.sh name1 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
for r in $(seq ${ROUNDS:-3}); do
  for v in base "$@"; do
    if [ $v = base ]; then unset ARSLAM_LIB; else export ARSLAM_LIB=ar_slam_amd/var_$v.so; fi
    timeout -k 10 300 python3 bench.py --config cfg5 --no-cpu-baseline --no-fingerprint > gpurun_out/loc_ab.json 2> gpurun_out/loc_ab.err || { tail gpurun_out/loc_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/loc_ab.json')); print(sys.argv[1], 'queries/s %.4g' % d['value'], 'kernel us %.1f' % d['roofline']['avg_launch_us'])" $v | tee -a gpurun_out/loc_ab.txt
  done
done
