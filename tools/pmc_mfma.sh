#!/bin/bash
# One PMC pass for the dominant kernel's MFMA utilisation (kernel trace only,
# no runtime/sys tracing): SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F64,
# SQ_BUSY_CYCLES, SQ_WAVE_CYCLES and GRBM_GUI_ACTIVE (the effective clock),
# over a short cfg3 bench; summary by tools/pmc_mfma.py.
# usage (on the box): bash tools/pmc_mfma.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d gpurun_out/pmcmfma_$tag -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-incremental --no-localize --no-kernel-timing --no-runtime-warmup \
  --no-fingerprint "$@" > gpurun_out/pmcmfma_$tag.log 2>&1 || exit $?
python3 tools/pmc_mfma.py gpurun_out/pmcmfma_$tag > gpurun_out/pmc_mfma_$tag.json
