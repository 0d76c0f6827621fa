"""Generate the committed golden fixtures from the CPU oracle (test infrastructure).

The reference's own tests pin nothing on this path, so the
fixtures are oracle outputs on seeded synthetic inputs:
  * jacobian_kat.npz  -- residual/Jacobian known-answer table (random draws incl.
                         w = 0 exactly and |w|^2 at DBL_EPSILON +- 0.1%),
                         cross-checked in tests against torch-fp64 autograd;
  * lm_<cfg>.json     -- LM traces (cost, radius, rho, step per iteration),
                         termination and final state summaries.
  * lm_ctl_<name>.json -- Ceres control-flow traces (CONTROL below): rejected
                         and invalid steps, every termination rule;
Usage: python tests/golden/make_golden.py [cfg ... | control | ctl_<name> ... | loc | kat]   (default: tiny small medium cfg2)
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


# Ceres control-flow traces: each names a graph (config
# + generator overrides) and solver options chosen so that one branch of the
# trust-region loop fires -- rejected steps (hard initial states, f0 = 3000,
# the reference default ar_slam_util.hpp:69), each termination rule, invalid
# steps through the forced-indefinite test hook, and FAILURE after more than
# max_num_consecutive_invalid_steps of them.
HARD = dict(init_trans_sigma=0.15, init_rot_sigma=0.25, f_init=3000.0)
HARD_M = dict(init_trans_sigma=0.12, init_rot_sigma=0.22, f_init=3000.0)
ALL_STEPS = 2 ** 64 - 1
CONTROL = {
    "tiny_reject": ("tiny", HARD, {}),
    "small_reject": ("small", HARD, {}),
    "medium_reject": ("medium", HARD_M, {}),
    "cfg2_reject": ("cfg2", HARD_M, {}),
    "small_min_radius": ("small", HARD, {"min_trust_region_radius": 100.0}),
    "small_max_iters": ("small", {}, {"max_num_iterations": 3}),
    "small_parameter": ("small", {}, {"function_tolerance": 0.0}),
    "medium_parameter": ("medium", {}, {"function_tolerance": 0.0}),
    "small_gradient": ("small", {}, {"function_tolerance": 0.0, "parameter_tolerance": 0.0,
                                     "gradient_tolerance": 1e-4}),
    "medium_gradient": ("medium", {}, {"function_tolerance": 0.0, "parameter_tolerance": 0.0,
                                       "gradient_tolerance": 1e-4}),
    "small_invalid": ("small", {}, {"debug_indefinite_mask": 0b110}),
    "medium_invalid": ("medium", {}, {"debug_indefinite_mask": 0b1010}),
    "tiny_failure": ("tiny", {}, {"debug_indefinite_mask": ALL_STEPS}),
    "small_failure": ("small", {}, {"debug_indefinite_mask": ALL_STEPS}),
}


def control_trace(name, threads=8):
    cfg, gkw, opts = CONTROL[name]
    g = synth.config_graph(cfg, **gkw)
    cam, cap, tag, s = O.solve_graph(g, num_threads=threads, **opts)
    its = s["iterations"]
    out = {"control": name, "config": cfg, "graph": gkw, "options": opts,
           "n_cap": g.n_cap, "n_tag": g.n_tag, "n_obs": g.n_obs,
           "termination": s["termination"], "rule": s["rule"],
           "num_linear_solves": s["num_linear_solves"],
           "num_successful_steps": s["num_successful_steps"],
           "num_unsuccessful_steps": s["num_unsuccessful_steps"],
           "initial_cost": s["initial_cost"], "final_cost": s["final_cost"], "final_focal": cam[0]}
    for k in ("cost", "cost_change", "trust_region_radius", "relative_decrease", "step_norm",
              "gradient_max_norm", "step_is_valid", "step_is_successful"):
        out[k] = [it[k] for it in its]
    # The same solve with no Schur elimination (the oracle's full normal
    # equations): a second exact arithmetic, whose distance from the Schur
    # trace measures how strongly this trajectory amplifies rounding.  The GPU
    # test allows the device a multiple of it (and never less than 1e-9).
    _, _, _, alt = O.solve_graph(g, num_threads=threads, elimination=1, **opts)
    assert [it["step_is_successful"] for it in alt["iterations"]] == out["step_is_successful"], name
    out["alt_cost"] = [it["cost"] for it in alt["iterations"]]
    out["alt_trust_region_radius"] = [it["trust_region_radius"] for it in alt["iterations"]]
    with open(os.path.join(HERE, f"lm_ctl_{name}.json"), "w") as f:
        json.dump(out, f, indent=1)


def map_yaml(g, uid=lambda c: f"cap_{c}", tag_id=lambda t: f"aruco_4X4_50_{t}", focal=3000.0):
    """A synthetic graph as a map file in the reference's layout (saveYaml ar_slam_util.cpp:387-465,
    SURVEY.md Appendix C): blocks in capture order, captures and arucos at zero pose (as detected,
    never solved: loadYaml leaves them uninitialized, :304-368), camera at the reference's default
    focal (CameraParams, ar_slam_util.hpp:68-72) and the demo's 1020x768 image."""
    blocks, arucos = [], {}
    for b in range(g.n_obs):
        t = int(g.obs_tag[b])
        arucos.setdefault(tag_id(t), {"pose": [0.0] * 6})
        blocks.append({"capture": uid(int(g.obs_cap[b])), "aruco": tag_id(t),
                       "aruco_rect": [float(v) for v in g.corners[b]]})
    captures = {uid(c): {"inv_pose": [0.0] * 6, "img_fn": f"img{c + 1}.jpg"} for c in range(g.n_cap)}
    return {"blocks": blocks, "captures": captures, "arucos": arucos,
            "camera": {"params": [focal, 0.0, 0.0], "width": synth.IMG_W, "height": synth.IMG_H}}


def cfg1_fixture():
    """cfg1 (BASELINE.json configs[0]): the demo's 3 captures / 6 tags as a detections map."""
    import yaml
    g = synth.config_graph("cfg1")
    with open(os.path.join(HERE, "cfg1_map.yaml"), "w") as f:
        f.write("# cfg1 replica: 3 captures / 6 tags, 1020x768, seed 16 (tests/golden/make_golden.py)\n")
        yaml.safe_dump(map_yaml(g), f, sort_keys=False, default_flow_style=None)


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
    if g.n_tag > 400:
        # the whole final state (camera, every capture and tag pose) of the large
        # configs: the trace above pins scalars only, this pins the parameters
        np.savez_compressed(os.path.join(HERE, f"lm_{name}_final.npz"), camera=cam, cap=cap, tag=tag,
                            final_cost=np.array(s["final_cost"]))


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
    ctl = list(CONTROL) if "control" in names else [n[4:] for n in names if n.startswith("ctl_")]
    for n in ctl:
        control_trace(n)
        print("wrote control", n)
    names = [n for n in names if n != "control" and not n.startswith("ctl_")]
    if "cfg1" in names:
        cfg1_fixture()
        print("wrote cfg1 map")
        names = [n for n in names if n != "cfg1"]
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
