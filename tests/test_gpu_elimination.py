"""GPU parity of the two elimination sides (arslam_lm_options.elimination).

DENSE_SCHUR eliminates Ceres' own e-block set (ar_slam_util.cpp:1011; Ceres
2.0 ComputeStableSchurOrdering): mostly tags on the demo-sized cfg1 graph and
early incremental graphs, mostly captures on the benchmark graphs.  The
device eliminates one whole side -- the majority side of that set under
ARSLAM_ELIM_AUTO -- by running its per-e-block kernels on the role-swapped
problem (captures become the reduced system).  Either side is the same exact
solve of the same LM system, so both must reproduce the oracle's trace
(capture elimination) to rounding: per-iteration cost 1e-9, final cost and
focal 1e-8, same termination, every gauge-aligned capture and tag pose
1e-6 m / 1e-7 rad (tests/gauge.py).
"""
import json
import os

import numpy as np
import pytest

from ar_slam_amd import synth
from gauge import assert_poses_match
from oracle.schur_ordering import ceres_e_blocks

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _compare(g, ours, ref):
    cam_o, cap_o, tag_o, s_o = ours
    cam_r, cap_r, tag_r, s_r = ref
    assert (s_o["termination"], s_o["rule"]) == (s_r["termination"], s_r["rule"])
    assert abs(len(s_o["iterations"]) - len(s_r["iterations"])) <= 1
    for a, b in list(zip([i["cost"] for i in s_o["iterations"]], [i["cost"] for i in s_r["iterations"]]))[:5]:
        assert abs(a - b) <= 1e-9 * abs(b)
    assert abs(s_o["final_cost"] - s_r["final_cost"]) <= 1e-8 * s_r["final_cost"]
    assert abs(cam_o[0] - cam_r[0]) <= 1e-8 * cam_r[0]
    assert_poses_match(cap_o, tag_o, cap_r, tag_r, tags=np.unique(g.obs_tag), caps=np.unique(g.obs_cap))


@pytest.mark.parametrize("side", ["captures", "tags", "auto"])
@pytest.mark.parametrize("name", ["cfg1", "tiny", "small", "medium", "wide"])
def test_both_sides_match_oracle(lm, oracle, name, side):
    g = synth.config_graph(name)
    elim = {"auto": lm.ELIM_AUTO, "captures": lm.ELIM_CAPTURES, "tags": lm.ELIM_TAGS}[side]
    ours = lm.solve_graph(g, elimination=elim)
    ref = oracle.solve_graph(g)
    _compare(g, ours, ref)
    s = ours[3]
    rule = ceres_e_blocks(g.obs_cap, g.obs_tag, g.n_cap, g.n_tag)
    assert (s["ceres_e_captures"], s["ceres_e_tags"]) == (rule["captures"], rule["tags"])
    if side == "auto":
        side = "tags" if rule["tags"] > rule["captures"] else "captures"
    assert s["elimination_used"] == {"captures": lm.ELIM_CAPTURES, "tags": lm.ELIM_TAGS}[side]
    # the reduced system is the other side plus the camera
    n_f = g.n_cap if side == "tags" else len(np.unique(g.obs_tag))
    assert s["n_reduced"] >= 6 * n_f + 1


@pytest.mark.parametrize("name", ["tiny_reject", "small_reject", "tiny_failure", "small_parameter"])
def test_control_traces_under_tag_elimination(lm, name):
    """Rejected steps, invalid steps -> FAILURE and the parameter rule, with tags eliminated."""
    with open(os.path.join(GOLDEN, f"lm_ctl_{name}.json")) as f:
        gold = json.load(f)
    g = synth.config_graph(gold["config"], **gold["graph"])
    opts = dict(gold["options"])
    mask = opts.pop("debug_indefinite_mask", 0)
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                            elimination=lm.ELIM_TAGS, **opts)
    rp.debug_force_indefinite(mask)
    s = rp.solve()
    its = s["iterations"]
    assert s["elimination_used"] == lm.ELIM_TAGS
    assert (s["termination"], s["rule"]) == (gold["termination"], gold["rule"])
    assert [it["step_is_valid"] for it in its] == gold["step_is_valid"]
    assert [it["step_is_successful"] for it in its] == gold["step_is_successful"]
    ours = np.array([it["cost"] for it in its])
    ref = np.array(gold["cost"])
    alt = np.array(gold["alt_cost"])
    tol = np.maximum(1e-9, 20.0 * np.abs(alt - ref) / np.abs(ref))
    assert np.all(np.abs(ours - ref) / np.abs(ref) <= tol)


def test_pointer_api_under_tag_elimination(lm):
    """Caller-owned blocks are written back to the right places when the device problem is
    role-swapped; re-solving reloads values only."""
    g = synth.config_graph("tiny")
    outs = []
    for elim in (lm.ELIM_CAPTURES, lm.ELIM_TAGS):
        camera = g.camera.copy()
        caps = [g.cap[c].copy() for c in range(g.n_cap)]
        tags = [g.tag[t].copy() for t in range(g.n_tag)]
        prob = lm.Problem(elimination=elim)
        for b in range(g.n_obs):
            prob.add_residual_block(g.corners[b], camera, caps[g.obs_cap[b]], tags[g.obs_tag[b]])
        s = prob.solve()
        assert s["elimination_used"] == elim
        s2 = prob.solve()   # from the solved state: values-only reload
        assert s2["setup_kind"] == lm.SETUP_VALUES
        outs.append((camera, np.stack(caps), np.stack(tags), s))
    (c1, k1, t1, s1), (c2, k2, t2, s2) = outs
    assert abs(s1["final_cost"] - s2["final_cost"]) <= 1e-9 * s1["final_cost"]
    np.testing.assert_allclose(c1, c2, rtol=1e-8)
    np.testing.assert_allclose(k1[:, :3] - k1[:, :3].mean(0), k2[:, :3] - k2[:, :3].mean(0), atol=1e-6)


def test_invalid_elimination_rejected(lm):
    g = synth.config_graph("tiny")
    with pytest.raises(lm.LMError):
        lm.solve_graph(g, elimination=7)
