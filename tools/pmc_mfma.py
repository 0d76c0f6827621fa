"""MFMA utilisation of k_factor_dag per launch from one rocprofv3 PMC pass (tools/pmc_mfma.sh).

mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x the launch's cycles), with the launch's
cycles from GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs; MI355X_MICROARCH.md, DVFS)
and, beside it, at the nominal 2.4 GHz over the kernel-trace duration.  MOPS_F64 x 512 = fp64
MFMA flops issued (16x16x4 f64: 2 x 16 x 16 x 4 = 2048 flops per wave-instruction, counted in
units of 512).  usage: pmc_mfma.py <dir>
"""
import collections
import csv
import glob
import json
import sys

KERNEL = "k_factor_dag"


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]


d = sys.argv[1]
acc = collections.defaultdict(list)
for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if short(r["Kernel_Name"]) == KERNEL:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = []
for path in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if short(r["Kernel_Name"]) == KERNEL:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
c = {k: sum(v) / len(v) for k, v in acc.items()}
mean_s = sum(dur) / len(dur) if dur else None
out = {"kernel": KERNEL, "launches": len(dur), "mean_us": mean_s * 1e6 if mean_s else None, "counters": c}
busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
gui = c.get("GRBM_GUI_ACTIVE")
if busy is not None and gui:
    out["effective_clock_ghz"] = gui / 8 / mean_s / 1e9 if mean_s else None
    out["mfma_busy_frac"] = busy / (1024 * gui / 8)
if busy is not None and mean_s:
    out["mfma_busy_frac_at_2p4ghz"] = busy / (1024 * mean_s * 2.4e9)
if "SQ_INSTS_VALU_MFMA_MOPS_F64" in c:
    out["mfma_f64_flops_per_launch"] = c["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
    if mean_s:
        out["mfma_f64_tflops"] = out["mfma_f64_flops_per_launch"] / mean_s / 1e12
out["note"] = __doc__.split("usage")[0].strip()
print(json.dumps(out, indent=1))
