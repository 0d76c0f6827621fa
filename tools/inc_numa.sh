#!/bin/bash
# The incremental cfg2 flow's full-load window (debug): a first process on the box (its memory cold),
# then warm processes with and without ARSLAM_SETUP_PROFILE.  usage: bash tools/inc_numa.sh
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
echo "numa_balancing: $(cat /proc/sys/kernel/numa_balancing 2>/dev/null)  thp: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null)"
for mode in prof prof; do
  if [ $mode = prof ]; then export ARSLAM_SETUP_PROFILE=1; else unset ARSLAM_SETUP_PROFILE; fi
  timeout -k 10 200 python3 tools/bench_incremental.py cfg2 > gpurun_out/incn.json 2> gpurun_out/incn.err || { tail gpurun_out/incn.err; exit 1; }
  echo "== $mode"; python3 -c "import json; d=json.load(open('gpurun_out/incn.json')); print('wall', round(d['wall_s'],3), 'setup', round(d['setup_ms_per_solve'],3), 'min', round(d['minimizer_ms_per_solve'],3), {k: v for k, v in d.items() if 'phase' in k})"
  [ $mode = prof ] && python3 tools/setup_summary.py gpurun_out/incn.err | grep -E "probe|setup "
done
exit 0
