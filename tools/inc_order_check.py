"""Debug: is the incremental flow's reused elimination order stale?  Runs
solveIncremental on cfg2 (as tools/bench_incremental.py), then loads the final
problem afresh (a new nested dissection) and compares the factorization plans
and the per-launch factorization time."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ar_slam_amd import build, lm, synth  # noqa: E402

build.build()
g = synth.config_graph(sys.argv[1] if len(sys.argv) > 1 else "cfg2")
s = lm.SlamSolver()
s.set_camera(g.camera)
for c in range(g.n_cap):
    sel = g.obs_cap == c
    s.add_detections(f"cap{c}", [f"tag_{t}" for t in g.obs_tag[sel]], g.corners[sel])
    s.solve_incremental()
last = s.last_summary()
caps, tags = s.capture_poses(), s.aruco_poses()
oc, ot, cr = [], [], []
for b in range(s.num_blocks):
    c, a, rect, added = s.block(b)
    if added:
        oc.append(c)
        ot.append(a)
        cr.append(rect)
cam = s.camera()[0]
out = {"incremental_last": {k: last[k] for k in ("n_factor_tiles", "n_levels", "factor_scalar_flops", "num_linear_solves")}}
out["incremental_last"]["factor_us_per_launch"] = 1e3 * last["t_cholesky_ms"] / max(last["num_linear_solves"], 1)
rp = lm.ResidentProblem(cam, caps, tags, np.array(oc, np.int32), np.array(ot, np.int32), np.array(cr), elimination=lm.ELIM_CAPTURES)
f = rp.solve()
out["fresh"] = {k: f[k] for k in ("n_factor_tiles", "n_levels", "factor_scalar_flops", "num_linear_solves")}
out["fresh"]["factor_us_per_launch"] = 1e3 * f["t_cholesky_ms"] / max(f["num_linear_solves"], 1)
print(json.dumps(out))
