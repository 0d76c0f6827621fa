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
wg = tr[:, 3] & 0xffffffff   # (column 3 holds the workgroup, not a time; debug flags above it)
flags = tr[:, 3] >> 32
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
cs = np.array(sorted(cont), int)
if len(cs):
    fl = flags[cs]
    print("continuations: premet %.2f  A_kk in D %.2f  fused tile prefetched %.2f" %
          tuple(np.mean((fl >> b) & 1) for b in range(3)))
    for b, nm in ((0, "premet"), (1, "A_kk in D")):
        for v in (1, 0):
            sel = cs[((fl >> b) & 1) == v]
            if len(sel):
                print(f"  {nm}={v} n={len(sel)} wait {np.mean(us[sel, 1] - us[sel, 0]):.2f} "
                      f"load+fold {np.mean(us[sel, 4] - us[sel, 1]):.2f}")
# the last POTRF tasks to finish (the root separators' chain): phases and flags
last = potrf[np.argsort(us[potrf, 2])][-int(sys.argv[2]) if len(sys.argv) > 2 else -24:]
print("   k   draw  +wait  +load  +potrf +publ  +trsm  +tail  flags(premet,AkkD,pref,next_met,claim) cont")
for t in last:
    u = us[t]
    print(f"{tasks[t, 1]:4d} {u[0]:6.1f} {u[1] - u[0]:5.2f} {u[4] - u[1]:6.2f} {u[5] - u[4]:6.2f} "
          f"{u[6] - u[5]:5.2f} {(u[7] - u[6]) if u[7] > 0 else 0:6.2f} {(u[2] - u[7]) if u[7] > 0 else u[2] - u[6]:6.2f}"
          f"   {int(flags[t]):05b}  {'c' if t in cont else '-'}")
# slack of the fused tile's late waits on that chain: when its last producer
# finished vs when the POTRF phase ended (negative: the solve waited for it)
nw = int(np.frombuffer(f.read(8), np.int64)[0])
woff = np.frombuffer(f.read(4 * (n + 1)), np.int32)
waits = np.frombuffer(f.read(8 * nw), np.int32).reshape(nw, 2)
sub = np.frombuffer(f.read(8 * n), np.int32).reshape(n, 2)
n_tiles = int(tasks[:, 3].max()) + 1
ready_prod, applied_prod = {}, {}
for t in range(n):
    ty, y, z, w = tasks[t]
    if ty in (0, 1):
        ready_prod[int(w)] = t
        if sub[t, 0] >= 0:
            ready_prod[int(sub[t, 0])] = t
    elif ty == 2:
        applied_prod.setdefault(int(w), []).append((int(z), t))
print("   k  potrf-end  late-ready  slack  (last late producer)")
for t in last:
    if sub[t, 0] < 0:
        continue
    best, who = -1e9, None
    for c, v in waits[sub[t, 1]:woff[t + 1]]:
        if c < n_tiles:
            u = ready_prod.get(int(c))
            if u is not None and u != t:
                tm = us[u, 7] if (tasks[u, 0] == 0 and sub[u, 0] == c) else (us[u, 6] if tasks[u, 0] == 0 else us[u, 2])
                if tm > best: best, who = tm, ("POTRF" if tasks[u, 0] == 0 else "TRSM", int(u))
        else:
            for s_, u in applied_prod.get(int(c) - n_tiles, []):
                if s_ < v and us[u, 2] > best: best, who = us[u, 2], ("UPD", int(u))
    print(f"{tasks[t, 1]:4d} {us[t, 5]:9.1f} {best:10.1f} {us[t, 5] - best:6.1f}  {who}")
