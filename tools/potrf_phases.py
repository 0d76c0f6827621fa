"""POTRF task phases from a DAG trace (ARSLAM_DAG_TRACE): per POTRF with a fused
TRSM, ready -> folded/loaded (t4), -> factored (t5), -> L_kk published (t6),
-> fused tile published (t7).  usage: potrf_phases.py trace.bin"""
import sys

import numpy as np

f = open(sys.argv[1], "rb")
n = int(np.frombuffer(f.read(8), np.int64)[0])
tasks = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
tr = np.frombuffer(f.read(64 * n), np.uint64).reshape(n, 8).astype(np.int64)
t0 = tr[:, 0].min()
us = lambda j: (tr[:, j] - t0) / 100.0
r, t4, t5, t6, t7, e = us(1), us(4), us(5), us(6), us(7), us(2)
p = (tasks[:, 0] == 0) & (tr[:, 7] > 0)
late = p & (r > np.percentile(r[p], 50))
for name, m in (("all fused POTRF", p), ("later half", late)):
    print(f"{name}: n={m.sum()}  fold/load {np.mean(t4[m]-r[m]):.2f}  potrf {np.mean(t5[m]-t4[m]):.2f}  "
          f"publish {np.mean(t6[m]-t5[m]):.2f}  fused {np.mean(t7[m]-t6[m]):.2f}  total {np.mean(t7[m]-r[m]):.2f} us")
