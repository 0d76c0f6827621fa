#!/bin/bash
# GPU test run on the box: tools/gpu_tests.sh <log name> [pytest args...]
# (default: the whole -m gpu suite); the log lands in gpurun_out/<name>.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
name=$1; shift
args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 900 python -u -m pytest "${args[@]}" -x -v --timeout 300 --timeout-method thread > gpurun_out/$name.txt 2>&1 || { tail -60 gpurun_out/$name.txt; exit 1; }
tail -3 gpurun_out/$name.txt
