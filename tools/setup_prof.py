"""Aggregate ARSLAM_SETUP_PROFILE lines of one incremental run (stderr file):
per line kind, count and total ms per phase.  usage: setup_prof.py <stderr file>"""
import collections
import re
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for line in open(sys.argv[1]):
    if not line.startswith("arslam "):
        continue
    head = line.split(":")[0] if ":" in line.split(" (")[0] else "arslam " + line.split()[1]
    cnt[head] += 1
    body = line[len(head) + 1:] if line.startswith(head + ":") else line[len("arslam "):]
    for name, val in re.findall(r"([a-z+_]+) ([0-9]+\.[0-9]+)", body):
        tot[head][name] += float(val)
for k in sorted(cnt):
    print(f"{k}: n={cnt[k]}", {n: round(v, 1) for n, v in tot[k].items()}, "ms total")
