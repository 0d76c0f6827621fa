#!/bin/bash
# build a variant library ar_slam_amd/var_<name>.so with extra compile flags (debug A/B)
# usage: bash tools/build_var.sh name "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/.."
ARSLAM_LIB=$PWD/ar_slam_amd/var_$1.so ARSLAM_EXTRA_FLAGS="$2" python -c "from ar_slam_amd import build; build.build(force=True)"
