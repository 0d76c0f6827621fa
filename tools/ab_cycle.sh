#!/bin/bash
# A/B on the box: bit-identity digests (tools/lib_cmp.py) of the default
# library and each variant ar_slam_amd/var_<name>.so, then the interleaved
# cfg3 A/B (tools/ab.py).  Optional: K=<pytest -k expr> runs those
# GPU tests first.  usage: bash tools/ab_cycle.sh name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
touch ar_slam_amd/*.so   # (built here: nothing on the box is rebuilt from a newer source mtime)
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/abt.log 2>&1 || { tail -40 gpurun_out/abt.log; exit 1; }
  tail -2 gpurun_out/abt.log
fi
timeout -k 10 200 python tools/lib_cmp.py cfg2 cfg3 > gpurun_out/cmp_default.txt 2>&1 || { tail gpurun_out/cmp_default.txt; exit 1; }
for v in "$@"; do
  ARSLAM_LIB=$PWD/ar_slam_amd/var_$v.so timeout -k 10 200 python tools/lib_cmp.py cfg2 cfg3 > gpurun_out/cmp_$v.txt 2>&1 || { tail gpurun_out/cmp_$v.txt; exit 1; }
  if cmp -s gpurun_out/cmp_default.txt gpurun_out/cmp_$v.txt; then echo "$v: bit-identical"; else echo "$v: DIFFERS"; paste gpurun_out/cmp_default.txt gpurun_out/cmp_$v.txt | head -4; fi
done
timeout -k 10 600 python -u tools/ab.py cfg3 3 base "$@"
