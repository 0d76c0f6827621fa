#!/bin/bash
# Time the panel kernel with parts removed (numerics are garbage in ablated runs).
export TMPDIR=/tmp
for ab in 0 1 2 4 8 16 31; do
  ARSLAM_PANEL_ABLATION=$ab timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$ab -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --skip-zero-tiles 1 --no-kernel-timing > gpurun_out/abl_$ab.log 2>&1 || exit 1
  echo "ablation $ab: $(python3 tools/kstats.py $(find gpurun_out/abl_$ab -name '*kernel_stats.csv') | grep k_panel)"
done
