"""Debug: single-process GPU LM trace vs the oracle on a named config (default medium)."""
import sys
sys.path.insert(0, '.')
import numpy as np
from ar_slam_amd import lm, synth
from oracle import oracle as O
name = sys.argv[1] if len(sys.argv) > 1 else "medium"
ex = int(sys.argv[2]) if len(sys.argv) > 2 else 1
g = synth.config_graph(name)
_, _, _, ref = O.solve_graph(g)
rp = lm.ResidentProblem(camera=g.camera, cap=g.cap, tag=g.tag, obs_cap=g.obs_cap, obs_tag=g.obs_tag,
                        corners=g.corners, device=0, factor_executor=ex)
s = rp.solve()
print(name, "gpu", s["termination"], s["rule"], len(s["iterations"]), "oracle", ref["termination"], ref["rule"], len(ref["iterations"]))
for a, b in zip(s["iterations"], ref["iterations"]):
    print(f"  {a['cost']:.12e} {b['cost']:.12e} valid {a.get('step_is_valid')} succ {a.get('step_is_successful')} r {a.get('trust_region_radius', 0):.3e}")
