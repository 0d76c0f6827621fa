"""POTRF phases of claimed continuations vs drawn POTRF tasks (debug; trace from
ARSLAM_DAG_TRACE).  A continuation runs on its predecessor's workgroup right
after it: drawn within 1 us of the end of a POTRF task on the same workgroup.
usage: potrf_cont.py trace.bin"""
import sys

import numpy as np

f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(64 * n), np.uint64).reshape(n, 8).astype(np.int64)
t0 = tr[:, 0].min()
us = (tr - t0) / 100.0
wg = tr[:, 3]   # (column 3 holds the workgroup, not a time)
potrf = np.where(tasks[:, 0] == 0)[0]
by_wg = {}
for t in np.argsort(us[:, 0]):
    by_wg.setdefault(int(wg[t]), []).append(int(t))
cont = set()
for lst in by_wg.values():
    for a, b in zip(lst, lst[1:]):
        if tasks[a, 0] == 0 and tasks[b, 0] == 0 and us[b, 0] - us[a, 2] < 1.0:
            cont.add(b)
for name, sel in (("continuation", [t for t in potrf if t in cont]), ("drawn", [t for t in potrf if t not in cont])):
    sel = np.array(sel, int)
    if not len(sel):
        continue
    ph = {"wait": us[sel, 1] - us[sel, 0], "load+fold": us[sel, 4] - us[sel, 1], "potrf": us[sel, 5] - us[sel, 4],
          "L_kk publish": us[sel, 6] - us[sel, 5], "fused trsm": us[sel, 7] - us[sel, 6], "tail": us[sel, 2] - us[sel, 7]}
    ok = us[sel, 7] > 0
    print(f"{name:13s} n={len(sel):4d} " + " ".join(
        f"{k} {np.mean(v[ok] if k in ('fused trsm', 'tail') else v):.2f}" for k, v in ph.items()))
