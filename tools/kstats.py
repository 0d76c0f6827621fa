"""Print a rocprofv3 kernel_stats.csv as a table (usage: kstats.py path [path...])."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== {path}  total {tot / 1e6:.3f} ms")
    for r in rows:
        print(f"{r['Name'][:58]:58s} {int(r['Calls']):7d} {float(r['TotalDurationNs']) / 1e3:11.1f} us"
              f" {float(r['AverageNs']) / 1e3:9.2f} us/call {100 * float(r['TotalDurationNs']) / tot:5.1f}%")
