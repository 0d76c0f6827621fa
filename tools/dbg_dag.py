import sys
import numpy as np
sys.path.insert(0, '.')
from ar_slam_amd import lm
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rng = np.random.default_rng(n)
B = rng.normal(size=(n, n))
A = B @ B.T + n * np.eye(n)
b = rng.normal(size=n)
L0, y0, i0 = lm.debug_dense_llt(A, b, executor=0)
print("level", n, i0, flush=True)
L1, y1, i1 = lm.debug_dense_llt(A, b, executor=1)
print("dag", n, i1, np.abs(L1 - L0).max(), np.abs(y1 - y0).max(), flush=True)
