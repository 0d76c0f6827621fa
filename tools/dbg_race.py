"""Debug: repeat the dense task-graph factorization of one SPD matrix and report
tiles whose bits differ between runs (a data race shows as varying bits)."""
import sys
import numpy as np
sys.path.insert(0, '.')
from ar_slam_amd import lm
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rng = np.random.default_rng(n)
B = rng.normal(size=(n, n))
A = B @ B.T + n * np.eye(n)
b = rng.normal(size=n)
L0, y0, i0 = lm.debug_dense_llt(A, b, executor=0)
runs = [lm.debug_dense_llt(A, b, executor=1) for _ in range(reps)]
T = (n + 1 + 63) // 64
for r, (L, y, info) in enumerate(runs):
    d = L != runs[0][0]
    bad = sorted({(i // 64, j // 64) for i, j in zip(*np.nonzero(d))})
    print(f"run {r}: info {info} |L-Llevel| {np.abs(L - L0).max():.2e} tiles differing from run 0: {len(bad)} {bad[:12]}",
          flush=True)
