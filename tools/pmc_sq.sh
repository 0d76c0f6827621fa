#!/bin/bash
# One PMC pass of SQ counters over a short cfg3 bench (kernel trace only).
# usage (on the box): bash tools/pmc_sq.sh <tag> "<counters>"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-trace -d gpurun_out/pmcsq_$1 -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 1 --warmup 0 > gpurun_out/pmcsq_$1.log 2>&1 || exit $?
python3 - "$1" <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in glob.glob(f"gpurun_out/pmcsq_{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k in ("k_schur", "k_linearize", "k_backsub", "k_schur_gather", "k_factor_dag"):
    if k in acc:
        print(k, {c: round(v / max(n[(k, c)], 1)) for c, v in acc[k].items()})
PY
