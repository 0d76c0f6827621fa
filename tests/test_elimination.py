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
