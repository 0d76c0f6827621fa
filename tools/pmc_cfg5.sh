#!/bin/bash
# PMC pass over the cfg5 localize bench (k_localize): VALU instruction count
# and wave-cycle breakdown -> gpurun_out/p5/pmc_localize.json
export TMPDIR=/tmp
OUT=gpurun_out/p5
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVES --kernel-trace -d $OUT/pmc -o run --output-format csv -- python3 bench.py --config cfg5 --no-cpu-baseline --steps 2 --warmup 0 > $OUT/pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections, json
acc = collections.defaultdict(float); n = collections.Counter()
for p in glob.glob('gpurun_out/p5/pmc/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'k_localize' in r['Kernel_Name']:
            acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
per = {k: v / n[k] for k, v in acc.items()}
json.dump({"note": "per k_localize launch (cfg5, 4096 queries); SQ_WAVE_CYCLES etc. in quad-cycles",
           "valu_instructions_per_launch": per.get("SQ_INSTS_VALU"), "counters": per},
          open('gpurun_out/p5/pmc_localize.json', 'w'), indent=1)
PY
