#!/bin/bash
# One GPU round trip: gpu tests, a short cfg3 bench, then the k_schur phase stamps
# (stamped rebuild).  Usage on the box: bash tools/gpu_cycle.sh [pytest-args]
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q ${@} > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phase_ms_per_solve'], d['roofline']['frac'])"
ARSLAM_EXTRA_FLAGS=-DARSLAM_SCHUR_STAMPS timeout -k 10 300 python ar_slam_amd/build.py --force > gpurun_out/bld.log 2>&1 || exit 1
timeout -k 10 120 python tools/schur_stamps.py 2>&1 | tail -2
timeout -k 10 300 python ar_slam_amd/build.py --force > gpurun_out/bld2.log 2>&1   # back to the unstamped library
