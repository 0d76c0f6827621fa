"""CPU tests of the e-block choice (ARSLAM_ELIM_AUTO) against the oracle's
restatement of Ceres 2.0's ComputeStableSchurOrdering
(oracle/schur_ordering.py): host logic only, no device.

ArSlamSolver::optimize asks for DENSE_SCHUR with no ordering
(ar_slam_util.cpp:1003-1012), so Ceres picks the e-blocks itself: the stable
greedy independent set of the Hessian graph in ascending degree.  On the
synthetic graphs of SURVEY.md §8d that is mostly captures (degree k+1 = 9
against a tag's ~28-41); on the demo-sized cfg1 graph and early incremental
graphs it is mostly tags.  Parity of that choice with Ceres itself is
unpinned (Ceres is not in the image).
"""
import numpy as np
import pytest

from ar_slam_amd import synth
from oracle.schur_ordering import ceres_e_blocks


@pytest.fixture(scope="module")
def L():
    from ar_slam_amd import build, lm
    build.build()
    return lm


def _both(L, g, **kw):
    ours = L.debug_ceres_e_blocks(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, **kw)
    ref = ceres_e_blocks(g.obs_cap, g.obs_tag, g.n_cap, g.n_tag, **kw)
    return ours, ref


@pytest.mark.parametrize("name", ["cfg1", "tiny", "small", "medium", "wide", "cfg2"])
def test_e_block_set_matches_restatement(L, name):
    g = synth.config_graph(name)
    ours, ref = _both(L, g)
    assert ours == ref


@pytest.mark.parametrize("name", ["tiny", "small"])
def test_e_block_set_with_constant_blocks(L, name):
    g = synth.config_graph(name)
    rng = np.random.default_rng(5)
    cap_const = (rng.random(g.n_cap) < 0.3).astype(np.uint8)
    tag_const = (rng.random(g.n_tag) < 0.3).astype(np.uint8)
    for kw in (dict(camera_const=True), dict(cap_const=cap_const), dict(tag_const=tag_const),
               dict(camera_const=True, cap_const=cap_const, tag_const=tag_const),
               dict(camera_const=True, tag_const=np.ones(g.n_tag, np.uint8))):
        ours, ref = _both(L, g, **kw)
        assert ours == ref, kw


def test_localize_problem_eliminates_every_capture(L):
    """localizeOne holds the camera and the map constant (ar_slam_util.cpp:965,972): every free
    block is a capture of degree 0, so Ceres eliminates all of them."""
    g = synth.config_graph("small")
    ours, _ = _both(L, g, camera_const=True, tag_const=np.ones(g.n_tag, np.uint8))
    assert ours["captures"] == g.n_cap and ours["tags"] == 0 and ours["camera"] == 0


def test_degenerate_graph_takes_the_camera(L):
    """One capture seeing one tag: camera, capture and tag all have degree 2; the camera comes
    first in program order, so Ceres' stable set is the camera alone."""
    ours = L.debug_ceres_e_blocks([900.0, 0, 0], np.zeros((1, 6)), np.zeros((1, 6)), [0], [0])
    assert ours == ceres_e_blocks([0], [0], 1, 1) == dict(captures=0, tags=0, camera=1, max_tag_obs=1)


def test_auto_side_by_config():
    """What AUTO eliminates (the majority side of Ceres' set): tags on the demo-sized graph,
    captures on the benchmark graphs."""
    for name, side in (("cfg1", "tags"), ("tiny", "tags"), ("medium", "captures"), ("cfg2", "captures")):
        g = synth.config_graph(name)
        r = ceres_e_blocks(g.obs_cap, g.obs_tag, g.n_cap, g.n_tag)
        got = "tags" if r["tags"] > r["captures"] else "captures"
        assert got == side, (name, r)


def test_invalid_problem_rejected(L):
    with pytest.raises(L.LMError):
        L.debug_ceres_e_blocks([900.0, 0, 0], np.zeros((1, 6)), np.zeros((1, 6)), [1], [0])


def _mixed_expected(g):
    m = ceres_e_blocks(g.obs_cap, g.obs_tag, g.n_cap, g.n_tag, members=True)
    ec, et = np.array(m["e_cap"], np.uint8), np.array(m["e_tag"], np.uint8)
    direct = len({int(c) for c, t in zip(g.obs_cap, g.obs_tag) if not ec[c] and not et[t]})
    return ec, et, direct


@pytest.mark.parametrize("name", ["cfg1", "small", "medium", "wide", "cfg2", "cfg2[:300]"])
def test_mixed_device_problem(L, name):
    """ELIM_MIXED regroups the residuals by Ceres' exact set: one group per eliminated capture
    and tag, one direct group per reduced-side capture with residuals joining two reduced-side
    poses; every other capture and tag is a reduced-side block."""
    g = synth.config_graph(name.split("[")[0])
    if "[:" in name:
        g = synth.prefix_graph(g, int(name.split("[:")[1][:-1]))
    r = L.debug_mixed_groups(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag)
    ec, et, direct = _mixed_expected(g)
    assert (r["e_cap"] == ec).all() and (r["e_tag"] == et).all()
    assert r["groups"] == ec.sum() + et.sum() + direct
    assert r["direct"] == direct
    assert r["f_blocks"] == g.n_cap + g.n_tag - ec.sum() - et.sum()


def test_incremental_prefixes_mix(L):
    """The reference's incremental flow on cfg2 solves mixed sets for most of its captures
    (captures and tags both eliminated from ~220 captures on)."""
    g = synth.config_graph("cfg2")
    kinds = []
    for k in (100, 300, 600, 1000):
        m = ceres_e_blocks(*(lambda h: (h.obs_cap, h.obs_tag, h.n_cap, h.n_tag))(synth.prefix_graph(g, k)))
        kinds.append((m["captures"] > 0, m["tags"] > 0))
    assert kinds == [(False, True), (True, True), (True, True), (True, True)]


@pytest.mark.parametrize("name", ["small", "medium", "wide"])
def test_oracle_mixed_set_matches_capture_elimination(name):
    """The oracle's DENSE_SCHUR over Ceres' mixed set (OR_ELIM_MIXED) is the same LM run as
    over the captures: the same exact step, rounding apart."""
    from oracle import oracle as O
    O.build()
    g = synth.config_graph(name)
    ec, et, _ = _mixed_expected(g)
    assert ec.sum() > 0 and et.sum() > 0
    a = O.solve_graph(g)[3]
    b = O.solve_graph(g, elimination=O.ELIM_MIXED, e_cap=ec, e_tag=et)[3]
    assert (a["termination"], a["rule"], len(a["iterations"])) == (b["termination"], b["rule"], len(b["iterations"]))
    for x, y in zip(a["iterations"], b["iterations"]):
        assert abs(x["cost"] - y["cost"]) <= 1e-11 * x["cost"]


def test_mixed_device_problem_with_constant_blocks(L):
    """Constant captures and tags are not in Ceres' graph: they stay on the reduced side (no
    rows), and residuals joining two reduced-side poses -- constant ones included -- go to the
    direct groups."""
    g = synth.config_graph("medium")
    rng = np.random.default_rng(11)
    cap_const = (rng.random(g.n_cap) < 0.1).astype(np.uint8)
    tag_const = (rng.random(g.n_tag) < 0.1).astype(np.uint8)
    r = L.debug_mixed_groups(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, cap_const=cap_const,
                             tag_const=tag_const)
    m = ceres_e_blocks(g.obs_cap, g.obs_tag, g.n_cap, g.n_tag, cap_const=cap_const, tag_const=tag_const,
                       members=True)
    ec, et = np.array(m["e_cap"], np.uint8), np.array(m["e_tag"], np.uint8)
    assert (r["e_cap"] == ec).all() and (r["e_tag"] == et).all()
    assert not (ec & cap_const).any() and not (et & tag_const).any()   # constants are never e-blocks
    direct = len({int(c) for c, t in zip(g.obs_cap, g.obs_tag) if not ec[c] and not et[t]})
    assert r["groups"] == ec.sum() + et.sum() + direct and r["direct"] == direct
    assert r["f_blocks"] == g.n_cap + g.n_tag - ec.sum() - et.sum()

