"""Sum the ARSLAM_SETUP_PROFILE lines of a run (debug): per kind, the count and the total of
every 'name value' millisecond field.  usage: setup_summary.py stderr.txt"""
import collections
import re
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for line in open(sys.argv[1]):
    m = re.match(r"arslam ([a-z_+]+):? (.*)", line.strip())
    if not m:
        continue
    kind, rest = m.group(1), m.group(2).split(" (")[0]
    cnt[kind] += 1
    toks = rest.replace(" ms", "").replace("gather plan", "gather_plan").split()
    if len(toks) == 1:
        tot[kind][kind] += float(toks[0])
        continue
    for a, b in zip(toks[::2], toks[1::2]):
        try:
            tot[kind][a] += float(b)
        except ValueError:
            pass
for k in tot:
    print(f"{k:12s} n={cnt[k]:5d} " + " ".join(f"{a} {v:.1f}" for a, v in tot[k].items() if a not in ("nc", "nt")) + " ms total")
