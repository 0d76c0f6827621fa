"""GPU busy time and idle gaps of a rocprofv3 kernel trace (debug): total kernel time, the
gaps between consecutive kernels bucketed by length, and the kernels that most often
follow a long gap (the host round trips of a host-driven loop).
usage: python tools/trace_gaps.py kernel_trace.csv[.gz]"""
import collections
import csv
import gzip
import sys

path = sys.argv[1]
op = gzip.open if path.endswith(".gz") else open
with op(path, "rt") as f:
    rows = list(csv.DictReader(f))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
busy = sum(e - s for s, e, _ in ks)
span = ks[-1][1] - ks[0][0]
print(f"kernels {len(ks)}  busy {busy / 1e6:.1f} ms  span {span / 1e6:.1f} ms  ({100 * busy / span:.1f} % busy)")
buckets = [(0, 2e3), (2e3, 5e3), (5e3, 10e3), (10e3, 20e3), (20e3, 50e3), (50e3, 200e3), (200e3, 1e12)]
tot = collections.Counter()
cnt = collections.Counter()
after = collections.Counter()
end = ks[0][1]
for s, e, n in ks[1:]:
    g = max(0, s - end)
    for b in buckets:
        if b[0] <= g < b[1]:
            tot[b] += g
            cnt[b] += 1
    if g >= 10e3:
        after[n] += 1
    end = max(end, e)
for b in buckets:
    print(f"gap {b[0] / 1e3:6.0f}-{b[1] / 1e3:6.0f} us: {cnt[b]:7d} gaps, {tot[b] / 1e6:8.1f} ms")
print("kernels after a gap >= 10 us:", after.most_common(8))
