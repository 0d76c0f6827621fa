#!/bin/bash
# default (host-direct scalars) full GPU suite; the MFMA-output k_schur variant's
# parity tests; digests and interleaved A/B of default, base, mfma
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ft.log 2>&1 || { tail -40 gpurun_out/ft.log; exit 1; }
tail -1 gpurun_out/ft.log
ARSLAM_LIB=$PWD/ar_slam_amd/var_mfma.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg3_matches_golden or both_sides or lm_solve_matches or control_trace or edge_cases or sharded_cfg3 or incremental_cfg2" > gpurun_out/ftm.log 2>&1 || { tail -40 gpurun_out/ftm.log; exit 1; }
tail -1 gpurun_out/ftm.log
bash tools/ab_cycle.sh base mfma
