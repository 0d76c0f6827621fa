#!/bin/bash
# Full GPU suite, then digests + interleaved A/B against the named variants.
# usage: bash tools/full_cycle.sh name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ft.log 2>&1 || { tail -40 gpurun_out/ft.log; exit 1; }
tail -2 gpurun_out/ft.log
bash tools/ab_cycle.sh "$@"
