"""Per-kernel HBM bytes per launch from two rocprofv3 PMC passes (tools/pmc_bench.sh).

FETCH_SIZE and WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE counts half the
bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM
section), so it is doubled; WRITE_SIZE is taken as is.  Both count
memory-side L2 requests, Infinity-Cache hits included.
usage: pmc_summary.py <prefix>   (reads <prefix>_FETCH_SIZE/, <prefix>_WRITE_SIZE/)
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(prefix, counter):
    acc = collections.defaultdict(lambda: [0.0, 0])
    for path in glob.glob(f"{prefix}_{counter}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
            acc[name][0] += float(r["Counter_Value"])
            acc[name][1] += 1
    return acc


prefix = sys.argv[1]
fetch = per_kernel(prefix, "FETCH_SIZE")
write = per_kernel(prefix, "WRITE_SIZE")
out = {"note": "bytes per launch; FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; KB -> bytes x1024",
       "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f, nf = fetch.get(k, [0.0, 0])
    w, nw = write.get(k, [0.0, 0])
    rd = 2 * f * 1024 / max(nf, 1)
    wr = w * 1024 / max(nw, 1)
    out["kernels"][k] = {"launches": max(nf, nw), "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                         "hbm_bytes_per_launch": rd + wr}
for name in ("k_factor_dag", "k_update"):   # persistent executor first, level launches otherwise
    dom = out["kernels"].get(name)
    if dom:
        out["dominant"] = name
        out["hbm_bytes_per_launch"] = dom["hbm_bytes_per_launch"]
        break
print(json.dumps(out, indent=1))
