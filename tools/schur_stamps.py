"""Diagnostic: per-phase cycles of k_schur (library built with -DARSLAM_SCHUR_STAMPS)."""
import ctypes as C
import sys
import numpy as np
sys.path.insert(0, '.')
from ar_slam_amd import lm, synth
g = synth.config_graph("cfg3")
rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, max_num_iterations=1)
s = rp.solve()
out = (C.c_ulonglong * 16)()
lm.lib().arslam_debug_schur_stamps(out)
v = np.array(out[:16], dtype=np.float64)
calls = s["num_linear_solves"]
print("k_schur calls", calls, "per-phase cycles per capture-wave:", np.round(v / (calls * g.n_cap)).astype(int).tolist())
