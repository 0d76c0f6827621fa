"""The gauge-aligned pose comparison the parity tests use (tests/gauge.py), on the CPU.

* A solution moved by any rigid motion compares equal to itself (the gauge is
  fitted away), for capture and tag positions and rotations.
* A capture pose written back to the wrong slot (what a wrong owner mapping in
  the sharded solve's write-back would do) fails, as does a rotation off by
  more than the tolerance.
"""
import numpy as np
import pytest

from ar_slam_amd import synth
from gauge import POS_TOL, ROT_TOL, assert_poses_match, pose_errors


def _moved(cap, tag, R, t):
    """The same map in another gauge x -> R x + t (see gauge.py)."""
    cap2, tag2 = cap.copy(), tag.copy()
    tag2[:, :3] = tag[:, :3] @ R.T + t
    tag2[:, 3:] = synth.log_so3(R[None] @ synth.rodrigues(tag[:, 3:]))
    cap2[:, :3] = -((-cap[:, :3]) @ R.T + t)
    cap2[:, 3:] = synth.log_so3(synth.rodrigues(cap[:, 3:]) @ R.T[None])
    return cap2, tag2


@pytest.fixture(scope="module")
def solved():
    g = synth.config_graph("small")
    return g.cap_true, g.tag_true


def test_gauge_motion_is_fitted_away(solved):
    cap, tag = solved
    R = synth.rodrigues(np.array([[0.3, -0.2, 0.5]]))[0]
    cap2, tag2 = _moved(cap, tag, R, np.array([1.0, -2.0, 0.5]))
    e = assert_poses_match(cap2, tag2, cap, tag)
    assert max(e.values()) < 1e-12, e


def test_misplaced_capture_fails(solved):
    cap, tag = solved
    bad = cap.copy()
    bad[[3, 7]] = bad[[7, 3]]   # two captures' poses swapped
    with pytest.raises(AssertionError):
        assert_poses_match(bad, tag, cap, tag)


def test_rotation_tolerance(solved):
    cap, tag = solved
    for scale, ok in ((0.2, True), (5.0, False)):
        t2 = tag.copy()
        w = synth.rodrigues(np.array([[0.0, 0.0, scale * ROT_TOL]]))[0]
        t2[4, 3:] = synth.log_so3(w[None] @ synth.rodrigues(tag[4:5, 3:]))[0]
        e = pose_errors(cap, t2, cap, tag)
        assert (e["tag_rot"] < ROT_TOL) == ok, e
        assert e["tag_pos"] < POS_TOL
