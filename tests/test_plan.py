"""CPU tests of the host-side symbolic analysis (arslam_debug_reduced_plan): the
reduced-system row layout and the tile Cholesky plan the solver would build,
without a device.

The layout restates ceres::Problem's parameter bookkeeping as ar_slam uses it
(ar_slam_util.cpp:720-727, 965, 972): a tag is a reduced parameter iff some
residual uses it and it is not constant; the camera likewise.  DENSE_SCHUR
eliminates the captures, so the reduced system has 6 rows per free tag and 3
for a free camera.
"""
import numpy as np
import pytest

from ar_slam_amd import synth


@pytest.fixture(scope="module")
def L():
    from ar_slam_amd import build, lm
    build.build()
    return lm


def _plan(L, g, **kw):
    return L.debug_reduced_plan(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, **kw)


@pytest.mark.parametrize("ordering", [0, 1, 2])
@pytest.mark.parametrize("name", ["small", "cfg2"])
def test_layout_rows_are_a_partition(L, name, ordering):
    g = synth.config_graph(name)
    info, tag_row = _plan(L, g, ordering=ordering)
    used = np.zeros(g.n_tag, bool)
    used[g.obs_tag] = True
    assert (tag_row[~used] == -1).all()            # unobserved tags are not parameters
    rows = np.concatenate([np.arange(r, r + 6) for r in tag_row[used]])
    assert len(np.unique(rows)) == rows.size      # 6 distinct rows per free tag
    assert info["camera_row"] == info["n_reduced"] - 3   # camera border last
    assert rows.max() < info["camera_row"]
    assert info["n_reduced"] == 6 * used.sum() + 3 + info["pad_rows"]
    assert info["n_padded"] % 64 == 0 and info["n_padded"] >= info["n_reduced"] + 1
    if ordering != 2:
        assert info["pad_rows"] == 0


def test_constant_blocks_have_no_rows(L):
    g = synth.config_graph("small")
    tag_const = np.zeros(g.n_tag, np.uint8)
    tag_const[::3] = 1
    info, tag_row = L.debug_reduced_plan(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                                         camera_const=True, tag_const=tag_const)
    assert (tag_row[::3] == -1).all()
    assert info["camera_row"] == -1
    info2, _ = L.debug_reduced_plan(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                                    camera_const=True, tag_const=np.ones(g.n_tag, np.uint8))
    assert info2["n_reduced"] == 0 and info2["n_levels"] == 0   # localize: nothing to factor


def test_dense_plan_flop_count(L):
    """Without zero-tile skipping the plan is the dense right-looking tile Cholesky."""
    g = synth.config_graph("small")
    info, _ = _plan(L, g, ordering=1, skip_zero_tiles=0)
    T = info["tiles_per_side"]
    assert info["n_factor_tiles"] == info["n_assembled_tiles"] == T * (T + 1) // 2
    assert info["n_levels"] == T
    t3 = 64.0 ** 3
    want = sum((T - k - 1) * 64 * 65 * 64 + (T - k - 1) * (T - k - 2) // 2 * 2 * t3 for k in range(T))
    assert info["update_flops"] == want


def test_nested_dissection_beats_band_on_cfg3(L):
    """Geometric nested dissection: a much shallower elimination tree than the RCM band."""
    g = synth.config_graph("cfg3")
    nd, _ = _plan(L, g, ordering=2)
    rcm, _ = _plan(L, g, ordering=1)
    assert nd["n_levels"] * 3 < rcm["n_levels"]
    assert nd["n_factor_tiles"] >= nd["n_assembled_tiles"]
    assert nd["pad_rows"] < 0.15 * nd["n_reduced"]   # separators absorb alignment padding
    again, _ = _plan(L, g, ordering=2)
    assert again == nd                               # deterministic


def test_invalid_problem_rejected_on_host(L):
    g = synth.config_graph("tiny")
    bad = g.obs_tag.copy()
    bad[0] = g.n_tag
    with pytest.raises(L.LMError):
        L.debug_reduced_plan(g.camera, g.cap, g.tag, g.obs_cap, bad, g.corners)


@pytest.mark.parametrize("name", ["medium", "cfg2", "cfg3"])
def test_task_graph_is_deadlock_free(L, name):
    """The persistent executor's ticket order: every wait is met by earlier tickets when run one at a
    time, and randomised interleavings of 1..512 concurrent workers never deadlock
    (dag_check / dag_simulate behind arslam_debug_reduced_plan)."""
    g = synth.config_graph(name)
    for ordering in (1, 2):
        info, _ = _plan(L, g, ordering=ordering)
        assert info["n_dag_tasks"] > 0
        assert info["dag_valid"] == 1, info
