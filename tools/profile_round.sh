#!/bin/bash
# Round profile of the cfg3 bench (and cfg5 localize) on the GPU box:
#   kernel trace + stats, then one PMC pass per counter group (rocprofv3 does
#   not split counters over passes; MI355X_MICROARCH.md block limits).
# usage (on the box): bash tools/profile_round.sh <out-dir under gpurun_out>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-incremental --steps 5 --warmup 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/stats.log 2>&1 || exit 11
for grp in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/pmc_$tag -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-incremental --no-kernel-timing --steps 2 --warmup 0 > $OUT/pmc_$tag.log 2>&1 || exit 12
done
L="python3 bench.py --config cfg5 --no-cpu-baseline --steps 5 --warmup 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/stats_cfg5 -o run --output-format csv -- $L > $OUT/stats_cfg5.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY --kernel-trace -d $OUT/pmc_cfg5_SQ -o run --output-format csv -- \
  python3 bench.py --config cfg5 --no-cpu-baseline --steps 2 --warmup 0 > $OUT/pmc_cfg5_SQ.log 2>&1 || exit 14
python3 tools/profile_summary.py $OUT > $OUT/summary.json
# keep only the summaries (gpurun copies back at most 64 MiB of gpurun_out/)
find $OUT -name "*kernel_trace.csv" -delete
find $OUT -name "*counter_collection.csv" -size +2M -delete
