"""Summarise a tools/profile_round.sh run: per-kernel launch count, mean duration
(rocprofv3 kernel trace), HBM bytes per launch (FETCH_SIZE x2 on gfx950 +
WRITE_SIZE, KB -> bytes; MI355X_MICROARCH.md HBM section) and the SQ counters
per launch.  usage: profile_summary.py <dir>"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]


def kname(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]


def trace(sub):
    acc = collections.defaultdict(list)
    for p in glob.glob(f"{d}/{sub}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            acc[kname(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    return {k: {"launches": len(v), "mean_us": sum(v) / len(v)} for k, v in acc.items()}


def pmc(sub):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    for p in glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            acc[kname(r)][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[kname(r)][r["Counter_Name"]] += 1
    return {k: {c: v / cnt[k][c] for c, v in cs.items()} for k, cs in acc.items()}


out = {"cfg3": trace("stats"), "cfg5": trace("stats_cfg5")}
fetch, write = pmc("pmc_FETCH_SIZE"), pmc("pmc_WRITE_SIZE")
for k in out["cfg3"]:
    f = fetch.get(k, {}).get("FETCH_SIZE")
    w = write.get(k, {}).get("WRITE_SIZE")
    if f is not None and w is not None:
        out["cfg3"][k]["hbm_bytes_per_launch"] = 2 * f * 1024 + w * 1024
sq = pmc("pmc_SQ_INSTS_VALU_MFMA_MOPS_F64")
for k, v in sq.items():
    if k in out["cfg3"]:
        out["cfg3"][k]["sq"] = v
for k, v in pmc("pmc_cfg5_SQ").items():
    if k in out["cfg5"]:
        out["cfg5"][k]["sq"] = v
print(json.dumps(out, indent=1))
