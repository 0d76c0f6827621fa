#!/bin/bash
# Round-3 re-entry check on the box: gpu tests, the cfg3 bench line, and SQ
# counter passes over the per-capture kernels (occupancy, VALU, LDS).
set -o pipefail
mkdir -p gpurun_out
bash tools/quick_cycle.sh || exit 1
bash tools/pmc_sq.sh occ "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM" || exit 1
