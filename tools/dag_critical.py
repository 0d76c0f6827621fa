"""Critical path of one persistent-executor factorization (debug; trace from ARSLAM_DAG_TRACE=path).

Walks back from the last task to finish: at each task the producer whose
completion came last is the predecessor.  Producers come from the task's
wait list (counter ready[tile] <- the POTRF/TRSM of that tile; counter
applied[tile] >= m <- the update items applying to that tile with sequence
number < m) plus, for an update item, the in-order apply wait on its own
target.  Each hop is split into
  run      the task's own execution (waits met -> end)
  draw     the task was drawn after its last producer finished (every
           workgroup busy, or the ticket order put it late)
  handoff  drawn in time, waits met later than the producer's end (counter
           visibility + spin granularity)
usage: dag_critical.py trace.bin
"""
import collections
import sys

import numpy as np

f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(64 * n), np.uint64).reshape(n, 8).astype(np.int64)
tr[:, 3] &= 0xffffffff   # (debug flags above the workgroup)
nw = int(np.frombuffer(f.read(8), np.int64)[0])
woff = np.frombuffer(f.read(4 * (n + 1)), np.int32)
waits = np.frombuffer(f.read(8 * nw), np.int32).reshape(nw, 2)
rest = f.read(8 * n)
sub = np.frombuffer(rest, np.int32).reshape(n, 2) if len(rest) == 8 * n else np.full((n, 2), -1, np.int32)
t0 = tr[:, 0].min()
us = lambda j: (tr[:, j] - t0) / 100.0   # s_memrealtime is 100 MHz
draw, ready, end = us(0), us(1), us(2)
pub_kk, pub_sub = us(6), us(7)   # POTRF: L_kk published; fused TRSM tile published
n_tiles = int(tasks[:, 3].max()) + 1
print(f"tasks {n}, makespan {end.max():.1f} us, workgroups {len(np.unique(tr[:, 3]))}")

ready_prod = {}
applied_prod = collections.defaultdict(list)   # tile -> [(seq, task)]
for t in range(n):
    ty, y, z, w = tasks[t]
    if ty in (0, 1):
        ready_prod[int(w)] = t
        if sub[t, 0] >= 0:
            ready_prod[int(sub[t, 0])] = t
    elif ty == 2:   # (INV tasks publish nothing another task waits for)
        applied_prod[int(w)].append((int(z), t))


def producers(t):
    """(producer task, time its awaited result was published)"""
    ps = []
    for c, v in waits[woff[t]:woff[t + 1]]:
        if c < n_tiles:
            if int(c) in ready_prod:
                u = ready_prod[int(c)]
                if tasks[u, 0] == 0:
                    ps.append((u, pub_sub[u] if sub[u, 0] == c else pub_kk[u]))
                else:
                    ps.append((u, end[u]))
        else:
            ps += [(u, end[u]) for s, u in applied_prod.get(int(c) - n_tiles, []) if s < v]
    ty, y, z, w = tasks[t]
    if ty == 2:   # in-order apply on the target
        ps += [(u, end[u]) for s, u in applied_prod.get(int(w), []) if s < z]
    return ps


path = []
seen = set()
t = int(np.argmax(end))
while True:
    path.append(t)
    seen.add(t)
    # a claimed POTRF publishes the tile it was claimed for: never walk back into the path itself
    ps = [p for p in producers(t) if p[0] not in seen]
    if not ps:
        break
    t = max(ps, key=lambda p: p[1])[0]
path.reverse()
names = ["POTRF", "TRSM", "UPD", "INV"]
acc = collections.defaultdict(float)
prev_end = draw[path[0]]
for t in path:
    ty = tasks[t, 0]
    acc[f"run {names[ty]}"] += end[t] - ready[t]
    acc["draw late"] += max(0.0, draw[t] - prev_end)
    acc["handoff"] += max(0.0, ready[t] - max(draw[t], prev_end))
    prev_end = end[t]
cnt = collections.Counter(names[tasks[t, 0]] for t in path)
print(f"critical path: {len(path)} tasks {dict(cnt)}, start {draw[path[0]]:.1f} us")
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"  {k:12s} {v:9.1f} us")
for ty, nm in enumerate(names):
    m = [t for t in path if tasks[t, 0] == ty]
    if m:
        r = np.array([end[t] - ready[t] for t in m])
        print(f"  {nm:6s} on path: n={len(m)} run mean {r.mean():.2f} us; all {nm}: run mean "
              f"{np.mean((end - ready)[tasks[:, 0] == ty]):.2f} us")
upd_on_path = [t for t in path if tasks[t, 0] == 2]
busy = np.sum(end - ready)
wgs = len(np.unique(tr[:, 3]))
print(f"busy {busy:.0f} us over {wgs} workgroups = {busy / wgs / end.max():.1%} of the makespan")
print("path:")
for t in path:
    ty, y, z, w = tasks[t]
    print(f"  {names[ty]:5s} ({y:5d},{z:5d}) draw {draw[t]:8.1f} ready {ready[t]:8.1f} end {end[t]:8.1f}")
