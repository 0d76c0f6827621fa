"""Debug: sub-phase times of the POTRF tasks of one executor trace
(ARSLAM_DAG_TRACE): waits met -> fold done -> potrf done -> L_kk published
-> fused TRSM published -> end, for the tile columns given (default: the
last 12 POTRFs to finish)."""
import sys
import numpy as np
f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(64 * n), np.uint64).reshape(n, 8).astype(np.int64)
t0 = tr[:, 0].min()
us = lambda t, j: (tr[t, j] - t0) / 100.0
po = np.nonzero(tasks[:, 0] == 0)[0]
sel = po[np.argsort(tr[po, 2])][-12:]
print("col    ready   fold  potrf  publ   sub(wait+trsm+publ)  rest")
for t in sel:
    r, a, b, c, d, e = us(t, 1), us(t, 4), us(t, 5), us(t, 6), us(t, 7), us(t, 2)
    sub = d - c if tr[t, 7] else float("nan")
    print(f"{tasks[t,1]:4d} {r:8.1f} {a-r:6.2f} {b-a:6.2f} {c-b:5.2f} {sub:8.2f} {e-(d if tr[t,7] else c):8.2f}")
