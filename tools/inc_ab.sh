#!/bin/bash
# Incremental cfg2 flow A/B on the box (debug): a warm-up process, then the default library and each
# variant ar_slam_amd/var_<name>.so (or env:NAME=VALUE[,NAME=VALUE], the default library under those switches) interleaved,
# ROUNDS times.  usage: ROUNDS=3 bash tools/inc_ab.sh name1 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
sha256sum ar_slam_amd/*.so | tee gpurun_out/inc_ab_libs.txt
timeout -k 10 200 python3 tools/bench_incremental.py cfg2 > /dev/null 2> gpurun_out/inc_ab.err || { tail gpurun_out/inc_ab.err; exit 1; }
for r in $(seq ${ROUNDS:-3}); do
  for v in base "$@"; do
    unset ARSLAM_LIB; envs=()
    case $v in base) ;; env:*) IFS=, read -ra envs <<< "${v#env:}" ;; *) export ARSLAM_LIB=ar_slam_amd/var_$v.so ;; esac
    timeout -k 10 200 env "${envs[@]}" python3 tools/bench_incremental.py cfg2 > gpurun_out/inc_ab.json 2> gpurun_out/inc_ab.err || { tail gpurun_out/inc_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/inc_ab.json')); print(sys.argv[1], 'wall %.3f setup %.3f min %.3f' % (d['wall_s'], d['setup_ms_per_solve'], d['minimizer_ms_per_solve']), d['load_setup_phase_ms'])" $v | tee -a gpurun_out/inc_ab.txt
  done
done
