#!/bin/bash
# rocprofv3 kernel stats of cfg3 (CFG=...) solves for the default library and variants (debug timing only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
touch ar_slam_amd/*.so
for v in base "$@"; do
  if [ $v = base ]; then unset ARSLAM_LIB; else export ARSLAM_LIB=$PWD/ar_slam_amd/var_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$v -o run --output-format csv -- python3 tools/ab.py --child ${CFG:-cfg3} 4 > gpurun_out/ks_$v.log 2>&1 || { tail gpurun_out/ks_$v.log; exit 1; }
  f=$(find gpurun_out/ks_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 tools/kstats.py "$f" | head -14; rm -rf gpurun_out/ks_$v
done
