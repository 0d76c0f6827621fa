#!/bin/bash
# usage (on the GPU box): tools/pmc_bench.sh <tag> [bench args...]
# Two separate PMC passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one
# TCC pass on gfx950), kernel trace only, no runtime/sys tracing.
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${tag}_$c -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-incremental --no-kernel-timing --no-runtime-warmup "$@" > gpurun_out/pmc_${tag}_$c.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_${tag} > gpurun_out/pmc_${tag}.json
