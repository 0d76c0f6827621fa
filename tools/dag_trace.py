"""Analyse a persistent-executor task timeline dumped with ARSLAM_DAG_TRACE=path (debug)."""
import sys
import numpy as np
f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(64 * n), np.uint64).reshape(n, 8).astype(np.int64)
tr[:, 3] &= 0xffffffff   # (debug flags above the workgroup)
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
sub = lambda j: (tr[:, j] - t0) / 100.0
for ty, name, labels in [(0, "POTRF", ["load+fold", "potrf", "store+release", "trinv+store"]),
                         (1, "TRSM", ["load", "trsm", "store+release"])]:
    m = tasks[:, 0] == ty
    pts = [ready] + [sub(j) for j in ([4, 5, 6] if ty == 0 else [4, 5])] + [end]
    print(name, " ".join(f"{lab} {np.mean(pts[i + 1][m] - pts[i][m]):.2f}" for i, lab in enumerate(labels)))
# POTRF chain timeline
m = np.nonzero(tasks[:, 0] == 0)[0]
o = m[np.argsort(ready[m])]
print("POTRF timeline (k, waits-met, end):")
for i in o[-25:]:
    print(f"  k={tasks[i,1]:4d} draw {draw[i]:8.1f} ready {ready[i]:8.1f} end {end[i]:8.1f}")
