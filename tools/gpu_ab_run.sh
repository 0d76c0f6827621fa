#!/bin/bash
# one box call (debug): interleaved A/B of the default library against variants on cfg3 and
# cfg2, then the -m gpu suite on the default library.  usage: bash tools/gpu_ab_run.sh v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
timeout -k 10 600 python -u tools/ab.py cfg3 ${ROUNDS:-3} base "$@" 2>&1 | tee gpurun_out/ab_cfg3.txt || exit 1
timeout -k 10 300 python -u tools/ab.py cfg2 2 base "$@" 2>&1 | tee gpurun_out/ab_cfg2.txt || exit 1
[ -n "$NOTEST" ] || bash tools/gpu_tests.sh gpu_tests_ab
