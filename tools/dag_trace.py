"""Analyse a persistent-executor task timeline dumped with ARSLAM_DAG_TRACE=path (debug)."""
import sys
import numpy as np
f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(32 * n), np.uint64).reshape(n, 4).astype(np.int64)
t0 = tr[:, 0].min()
draw, ready, end = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, (tr[:, 2] - t0) / 100.0   # 100 MHz -> us
print(f"tasks {n}, makespan {end.max():.1f} us, workgroups {len(np.unique(tr[:, 3]))}")
for ty, name in enumerate(["POTRF", "TRSM", "UPD"]):
    m = tasks[:, 0] == ty
    if m.any():
        print(f"{name:6s} n={m.sum():6d} wait mean {np.mean(ready[m]-draw[m]):7.2f} us  run mean {np.mean(end[m]-ready[m]):7.2f} "
              f"max {np.max(end[m]-ready[m]):7.2f}  total run {np.sum(end[m]-ready[m]):9.1f}")
busy = np.sum(end - ready)
print(f"sum(run) {busy:.1f} us over {len(np.unique(tr[:, 3]))} WGs -> {busy / len(np.unique(tr[:, 3])):.1f} us each; "
      f"sum(wait) {np.sum(ready - draw):.1f}")
# POTRF chain timeline
m = np.nonzero(tasks[:, 0] == 0)[0]
o = m[np.argsort(ready[m])]
print("POTRF timeline (k, waits-met, end):")
for i in o[-25:]:
    print(f"  k={tasks[i,1]:4d} draw {draw[i]:8.1f} ready {ready[i]:8.1f} end {end[i]:8.1f}")
