"""Generate the committed golden fixtures from the CPU oracle (test infrastructure).

The reference's own tests pin nothing on this path, so the
fixtures are oracle outputs on seeded synthetic inputs:
  * jacobian_kat.npz  -- residual/Jacobian known-answer table (random draws incl.
                         w = 0 exactly and |w|^2 at DBL_EPSILON +- 0.1%),
                         cross-checked in tests against torch-fp64 autograd;
  * lm_<cfg>.json     -- LM traces (cost, radius, rho, step per iteration),
                         termination and final state summaries.
Usage: python tests/golden/make_golden.py [cfg ...]   (default: tiny small medium cfg2)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from ar_slam_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

EPS = np.finfo(float).eps


def jacobian_kat(n=256, seed=5):
    rng = np.random.default_rng(seed)
    cam = np.stack([rng.uniform(500, 3000, n), np.zeros(n), np.zeros(n)], 1)
    tag = np.concatenate([rng.normal(0, 1, (n, 3)), rng.normal(0, 1, (n, 3))], 1)
    w = rng.normal(0, 1, (n, 3))
    scale = np.ones(n)
    scale[0::8] = 0.0
    scale[1::8] = 1e-2
    scale[2::8] = 3.0
    w = w * scale[:, None]
    for i in range(3, n, 8):
        w[i] *= np.sqrt(EPS) * (0.999 if (i // 8) % 2 else 1.001) / np.linalg.norm(w[i])
    cap = np.concatenate([-tag[:, :3] + rng.normal(0, 0.2, (n, 3)) + [0, 0, 1.0], w], 1)
    tag[4::8, 3:] = 0.0
    corners = rng.normal(0, 100, (n, 8))
    r = np.zeros((n, 8))
    J = np.zeros((n, 8, 15))
    for i in range(n):
        r[i], J[i] = O.residual_jacobian(cam[i], cap[i], tag[i], corners[i])
    np.savez_compressed(os.path.join(HERE, "jacobian_kat.npz"), cam=cam, cap=cap, tag=tag,
                        corners=corners, r=r, J=J)


def lm_trace(name, threads=8):
    g = synth.config_graph(name)
    cam, cap, tag, s = O.solve_graph(g, num_threads=threads)
    its = s["iterations"]
    out = {
        "config": name, "n_cap": g.n_cap, "n_tag": g.n_tag, "n_obs": g.n_obs,
        "termination": s["termination"], "rule": s["rule"],
        "num_linear_solves": s["num_linear_solves"],
        "initial_cost": s["initial_cost"], "final_cost": s["final_cost"],
        "cost": [it["cost"] for it in its],
        "trust_region_radius": [it["trust_region_radius"] for it in its],
        "relative_decrease": [it["relative_decrease"] for it in its],
        "step_norm": [it["step_norm"] for it in its],
        "gradient_max_norm": [it["gradient_max_norm"] for it in its],
        "step_is_successful": [it["step_is_successful"] for it in its],
        "final_focal": cam[0],
        "final_rms_px": synth.rms_px(s["final_cost"], g.n_obs),
        # gauge-invariant summary of the final map: pairwise tag-centre distances
        "tag_xyz_final": tag[:, :3].tolist() if g.n_tag <= 400 else None,
    }
    with open(os.path.join(HERE, f"lm_{name}.json"), "w") as f:
        json.dump(out, f, indent=1)


def localize_golden(n_query=4096):
    """cfg5: localizeMany (ar_slam_util.cpp:888-979) of n_query queries against cfg3's map."""
    b = synth.make_localize_batch(n_query=n_query)
    pose, status, sums = O.localize_many(b, with_summaries=True)
    np.savez_compressed(os.path.join(HERE, "loc_cfg5.npz"), pose=pose, status=status,
                        initial_cost=np.array([s["initial_cost"] for s in sums]),
                        final_cost=np.array([s["final_cost"] for s in sums]),
                        n_iters=np.array([len(s["iterations"]) for s in sums], np.int32),
                        rule=np.array([s["rule"] for s in sums]))


if __name__ == "__main__":
    names = sys.argv[1:] or ["tiny", "small", "medium", "cfg2"]
    if "loc" in names:
        localize_golden()
        print("wrote loc")
        names = [n for n in names if n != "loc"]
    if "kat" in names or not sys.argv[1:]:
        jacobian_kat()
    for n in names:
        if n != "kat":
            lm_trace(n)
            print("wrote", n)
