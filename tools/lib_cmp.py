"""Debug: one resident solve per config with the library ARSLAM_LIB names; prints
a digest of the iteration trace and the final parameters, so two variant
builds that must be bit-identical can be compared line by line.
usage: ARSLAM_LIB=... python tools/lib_cmp.py [config ...]"""
import hashlib
import sys

import numpy as np

sys.path.insert(0, ".")
from ar_slam_amd import lm, synth  # noqa: E402

for name in sys.argv[1:] or ["cfg2", "cfg3"]:
    g = synth.config_graph(name)
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, phase_timing=0)
    h = hashlib.sha1()
    for _ in range(2):
        s = rp.solve()
        h.update(np.array([i["cost"] for i in s["iterations"]], np.float64).tobytes())
    for a in (rp.camera, rp.cap, rp.tag):
        h.update(np.ascontiguousarray(a).tobytes())
    print(name, len(s["iterations"]), s["final_cost"], h.hexdigest()[:16], flush=True)
