#!/bin/bash
# A/B on the box (debug): interleaved cfg solves of the default library and variants
# ar_slam_amd/var_<name>.so (tools/ab.py).  usage: CFG=cfg3 ROUNDS=3 bash tools/ab.sh name1 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so   # (built here: nothing on the box is rebuilt from a newer source mtime)
sha256sum ar_slam_amd/*.so | tee gpurun_out/ab_libs.txt
timeout -k 10 900 python -u tools/ab.py ${CFG:-cfg3} ${ROUNDS:-3} base "$@" 2>&1 | tee gpurun_out/ab.txt
