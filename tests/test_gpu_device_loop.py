"""The device-resident LM loop (lm_device.hip) against the host loop.

Both loops run the same kernels on the same data; only the place where
Ceres' step decisions are taken differs (TrustRegionMinimizer's step
evaluation and FinalizeIterationAndCheckIfMinimizerCanContinue restated in
k_lm_decide / k_lm_finalize, lm_solver.hip's host loop otherwise; SURVEY.md
Appendix B).  The traces must therefore agree bit for bit: every recorded
cost, radius, step validity and success, the termination rule, the step
count and the final parameters.  The control traces (tests/golden/lm_ctl_*)
cover rejected steps, invalid steps (the forced-indefinite hook), FAILURE
after consecutive invalid steps and every termination rule.
"""
import glob
import json
import os

import numpy as np
import pytest

from ar_slam_amd import synth

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CONTROL = sorted(os.path.basename(p)[7:-5] for p in glob.glob(os.path.join(GOLDEN, "lm_ctl_*.json")))
KEYS = ("cost", "trust_region_radius", "step_is_valid", "step_is_successful", "relative_decrease",
        "gradient_max_norm", "step_norm", "cost_change")


@pytest.fixture(scope="module")
def lm():
    from ar_slam_amd import build, lm as L
    build.build()
    return L


def _solve(lm, g, device_loop, mask=0, **opts):
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                            device_loop=device_loop, phase_timing=0, **opts)
    rp.debug_force_indefinite(mask)
    s = rp.solve()
    return s, rp.camera.copy(), rp.cap.copy(), rp.tag.copy()


def _same(a, b):
    sa, ca, xa, ta = a
    sb, cb, xb, tb = b
    assert (sa["termination"], sa["rule"]) == (sb["termination"], sb["rule"])
    assert sa["num_linear_solves"] == sb["num_linear_solves"]
    assert sa["num_successful_steps"] == sb["num_successful_steps"]
    assert sa["num_unsuccessful_steps"] == sb["num_unsuccessful_steps"]
    assert len(sa["iterations"]) == len(sb["iterations"])
    for ia, ib in zip(sa["iterations"], sb["iterations"]):
        assert ia["iteration"] == ib["iteration"]
        for k in KEYS:
            assert ia[k] == ib[k], (ia["iteration"], k, ia[k], ib[k])
    assert sa["final_cost"] == sb["final_cost"]
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(xa, xb)
    np.testing.assert_array_equal(ta, tb)


@pytest.mark.parametrize("name", CONTROL)
def test_control_trace_device_loop_matches_host_loop(lm, name):
    with open(os.path.join(GOLDEN, f"lm_ctl_{name}.json")) as f:
        gold = json.load(f)
    g = synth.config_graph(gold["config"], **gold["graph"])
    opts = dict(gold["options"])
    mask = opts.pop("debug_indefinite_mask", 0)
    host = _solve(lm, g, 0, mask, **opts)
    dev = _solve(lm, g, 1, mask, **opts)
    assert host[0]["lm_loop"] == lm.LOOP_HOST
    assert dev[0]["lm_loop"] in (lm.LOOP_DEVICE, lm.LOOP_GRAPH)
    _same(host, dev)


@pytest.mark.parametrize("name", ["medium", "cfg2", "cfg3"])
def test_device_loop_matches_host_loop(lm, name):
    g = synth.config_graph(name)
    host = _solve(lm, g, 0)
    dev = _solve(lm, g, 1)
    assert dev[0]["lm_loop"] == lm.LOOP_GRAPH
    _same(host, dev)


def test_device_loop_dominant_kernel_timing(lm):
    """kernel_timing inside the captured iterations: one k_factor_dag duration per linear solve
    (the iterations enqueued past the end return at their gates and are not counted)."""
    g = synth.config_graph("cfg2")
    s, *_ = _solve(lm, g, 1, kernel_timing=1)
    assert s["lm_loop"] == lm.LOOP_GRAPH
    assert s["n_dominant_launches"] == s["num_linear_solves"]
    assert s["t_dominant_ms"] > 0.0


def test_device_loop_resolves_and_reuses_its_graphs(lm):
    """Repeated solves of the resident problem (the bench's step) give identical traces."""
    g = synth.config_graph("cfg2")
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, phase_timing=0,
                            device_loop=1)
    a = rp.solve()
    b = rp.solve()
    assert a["lm_loop"] == b["lm_loop"] == lm.LOOP_GRAPH
    assert [i["cost"] for i in a["iterations"]] == [i["cost"] for i in b["iterations"]]


def test_host_loop_when_a_callback_needs_every_iteration(lm):
    """An iteration callback (or per-iteration write-back, progress output, phase timing) keeps
    the host loop: the host acts between iterations."""
    g = synth.config_graph("small")
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, phase_timing=0,
                            device_loop=1)
    seen = []
    rp.set_iteration_callback(lambda it: (seen.append(it["iteration"]), 0)[1])
    s = rp.solve()
    assert s["lm_loop"] == lm.LOOP_HOST
    assert seen == [i["iteration"] for i in s["iterations"]]
    rp2 = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, phase_timing=1,
                            device_loop=1)
    assert rp2.solve()["lm_loop"] == lm.LOOP_HOST
