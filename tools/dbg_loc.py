import sys
import numpy as np
sys.path.insert(0, '.')
from ar_slam_amd import lm, synth
from oracle import oracle as O
b = synth.make_localize_batch(n_query=512)
pose, res = lm.localize_many(b)
pose_o, st, sums = O.localize_many(b, with_summaries=True)
for q in (10, 19):
    print("query", q, "gpu:", {k: res[k][q] for k in ("status", "rule", "num_iterations", "num_successful_steps", "num_unsuccessful_steps", "initial_cost", "final_cost")})
    s = sums[q]
    print("  oracle:", s["termination"], s["rule"], s["initial_cost"], s["final_cost"], s["num_successful_steps"], s["num_unsuccessful_steps"])
    for it in s["iterations"]:
        print("   ", it["iteration"], repr(it["cost"]), it["cost_change"], it["relative_decrease"], it["trust_region_radius"], it["step_is_successful"], it["step_norm"])
    print("  pose diff", pose[q] - pose_o[q])
