#!/bin/bash
# GPU suite (multirank included), then the list-schedule cost sweep and the incremental flow.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/qt.log 2>&1 || { tail -40 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
bash tools/sim_sweep.sh "$@" || exit 1
ARSLAM_SETUP_PROFILE=1 timeout -k 10 200 python tools/bench_incremental.py cfg2 > gpurun_out/inc.log 2> gpurun_out/inc.err || { tail -5 gpurun_out/inc.err; exit 1; }
tail -3 gpurun_out/inc.log
