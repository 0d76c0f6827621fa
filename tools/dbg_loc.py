import numpy as np, sys
sys.path.insert(0, '.')
from ar_slam_amd import lm, synth
g = synth.config_graph("medium")
tag_const = np.ones(g.n_tag, np.uint8)
ours = lm.solve_soa(g.camera_true.copy(), g.cap, g.tag_true, g.obs_cap, g.obs_tag, g.corners, camera_const=True, tag_const=tag_const)
s = ours[3]
print({k: v for k, v in s.items() if k != 'iterations'})
for it in s['iterations'][:8]: print(it)
