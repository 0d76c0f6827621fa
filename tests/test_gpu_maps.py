"""GPU tests of the map-file flow and of cfg1 (BASELINE.json configs[0]).

* Map file -> device solve -> map file (§8f row 3): loadYaml
  (ar_slam_util.cpp:304-368) of a map in the reference's layout, solve()
  (the BFS driver, :744-866, every optimize() a device solve through the
  C-ABI), saveYaml (:387-465); the result is compared with the oracle's
  restatement of the same driver (oracle/driver.py) on the same map, and the
  saved file is read back with PyYAML and must hold the device's state
  exactly.  This is the ar_slam_cli flow (ar_slam_cli.cpp:51-78).
* cfg1: the demo's 3 captures / 6 tags (demo_launch.py:39-110), as a
  committed synthetic detections fixture (tests/golden/cfg1_map.yaml, made
  by make_golden.py: real detections need OpenCV's ArUco dictionaries, absent
  from the image), fed one Detections message at a time with a
  solveIncremental after each (the ROS node's flow, :629-742).

Tolerances (tests/spread_tol.py): as tests/test_gpu_slam.py (a chain of full
solves: costs and focal 1e-6 relative; poses as tag and camera centres after
a rigid alignment, 1e-5 m), widened to 20x the distance between the oracle's
own Schur and full-normal-equation runs of the same driver where the problem
itself amplifies rounding, but capped at focal 1e-3 px, centres 1e-4 m, cost
1e-6 relative.  Three values are exempt from the caps, each with its reason
asserted (spread_tol.EXEMPT): cfg1's first message is one capture of 4 tags
with no fixed block, which Ceres' LM leaves at NO_CONVERGENCE after 50
iterations in a flat valley, where two exact arithmetics already differ by
2e-5 in cost and 5e-2 px in focal, and the second message inherits that
focal drift.  The gauge-invariant reprojection RMS of every converged cfg1
solve (the map file and the final message) agrees to 1e-8 relative.
"""
import os

import numpy as np
import pytest

from ar_slam_amd import synth
from spread_tol import tolerance

pytestmark = pytest.mark.gpu
yaml = pytest.importorskip("yaml")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _messages(doc):
    """Detections per capture, in the file's capture order (blocks are capture-major)."""
    rects = {}
    for b in doc["blocks"]:
        rects.setdefault(b["capture"], []).append((b["aruco"], b["aruco_rect"]))
    for uid in doc["captures"]:
        ids = [a for a, _ in rects.get(uid, [])]
        yield uid, ids, np.array([r for _, r in rects.get(uid, [])], np.float64).reshape(-1, 8)


def _state(o):
    return (o.last_summary["final_cost"], o.camera[0], np.array([c["pose"] for c in o.captures]),
            np.array([a["pose"] for a in o.arucos]))


def _align_rigid(P, Q):
    """Rigid (Kabsch) alignment of point sets P -> Q; returns aligned P."""
    pc, qc = P.mean(0), Q.mean(0)
    U, _, Vt = np.linalg.svd((P - pc).T @ (Q - qc))
    d = np.sign(np.linalg.det(Vt.T @ U.T))
    R = Vt.T @ np.diag([1, 1, d]) @ U.T
    return (R @ (P - pc).T).T + qc


def _points(caps, tags):
    """Gauge-covariant points: tag centres and camera centres (-t_c of the inverse pose)."""
    return np.concatenate([np.asarray(tags)[:, :3], -np.asarray(caps)[:, :3]])


def _compare(s, o, alt, key=None, rms_rel=None):
    """Device vs oracle `o`; `alt` is the oracle run with the full normal equations.  Costs and
    focal directly; poses as tag and camera centres after a rigid alignment onto the oracle's
    (no block is held constant: the solution is defined up to a rigid motion, and the flat
    first solve leaves the gauge wherever the rounding took it).  Tolerances: spread_tol (the
    oracle's two arithmetics' spread, capped; key = (flow, message) for the named exemptions);
    rms_rel: the reprojection RMS (gauge-invariant) to that relative tolerance as well."""
    assert s.num_solves == o.n_solves == alt.n_solves
    last = s.last_summary()
    assert last["termination"] == o.last_summary["termination"]
    ref, oth = _state(o), _state(alt)
    ours = (last["final_cost"], s.camera()[0][0])
    for what, a, b, c in zip(("cost", "focal"), ours, ref, oth):
        tol = tolerance(what, b, c, key)
        assert abs(a - b) <= tol, (what, key, a, b, tol)
    q = _points(ref[2], ref[3])
    p_ours = _align_rigid(_points(s.capture_poses(), s.aruco_poses()), q)
    p_alt = _align_rigid(_points(oth[2], oth[3]), q)
    tol = np.vectorize(lambda qq, aa: tolerance("centres", qq, aa, key))(q, p_alt)
    assert np.all(np.abs(p_ours - q) <= tol), ("centres", key, np.max(np.abs(p_ours - q)), np.max(np.abs(p_alt - q)))
    if rms_rel is not None:   # (final_rms_px = sqrt(2 cost / (4 n_obs)), synth.rms_px)
        rms_ref = synth.rms_px(ref[0], last["n_obs"])
        assert abs(last["final_rms_px"] - rms_ref) <= rms_rel * rms_ref, ("rms", key, last["final_rms_px"], rms_ref)


def _write_map(g, path):
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import map_yaml
    doc = map_yaml(g, focal=float(g.camera[0]))   # (from f = 3000 the BFS chain on `small` is chaotic:
    with open(path, "w") as f:                    #  the oracle's two arithmetics land metres apart)
        yaml.safe_dump(doc, f, sort_keys=False, default_flow_style=None)
    return doc


@pytest.mark.parametrize("name", ["cfg1", "tiny", "small"])
def test_map_file_solve_save_matches_oracle(lm, name, tmp_path):
    from oracle.driver import OracleSlam
    if name == "cfg1":
        path = os.path.join(GOLDEN, "cfg1_map.yaml")
        with open(path) as f:
            doc = yaml.safe_load(f)
    else:
        path = str(tmp_path / "map.yaml")
        doc = _write_map(synth.config_graph(name), path)
    s = lm.SlamSolver()
    s.load_yaml(path)
    assert (s.num_captures, s.num_blocks) == (len(doc["captures"]), len(doc["blocks"]))
    s.solve()
    o = OracleSlam(camera=doc["camera"]["params"])
    alt = OracleSlam(camera=doc["camera"]["params"], elimination=1)
    for x in (o, alt):
        for uid, ids, corners in _messages(doc):
            x.add_detections(uid, ids, corners)
        x.solve()
    _compare(s, o, alt, rms_rel=1e-8 if name == "cfg1" else None)
    assert s.last_summary()["final_rms_px"] < 1.0
    out = tmp_path / "solved.yaml"
    s.save_yaml(out)
    with open(out) as f:
        saved = yaml.safe_load(f)
    assert list(saved["captures"]) == list(doc["captures"])
    np.testing.assert_array_equal(np.array([saved["captures"][u]["inv_pose"] for u in saved["captures"]]),
                                  s.capture_poses())
    ids = [s.aruco(a)[0] for a in range(s.num_arucos)]
    np.testing.assert_array_equal(np.array([saved["arucos"][i]["pose"] for i in ids]), s.aruco_poses())
    assert saved["camera"]["params"] == list(s.camera()[0])
    assert (saved["camera"]["width"], saved["camera"]["height"]) == (synth.IMG_W, synth.IMG_H)
    assert [b["aruco_rect"] for b in saved["blocks"]] == [b["aruco_rect"] for b in doc["blocks"]]


def test_cfg1_incremental_messages_match_oracle(lm):
    """cfg1 through the ROS node's flow: addDetections + solveIncremental per message."""
    from oracle.driver import OracleSlam
    with open(os.path.join(GOLDEN, "cfg1_map.yaml")) as f:
        doc = yaml.safe_load(f)
    s = lm.SlamSolver()
    o = OracleSlam(camera=doc["camera"]["params"])
    alt = OracleSlam(camera=doc["camera"]["params"], elimination=1)
    s.set_camera(doc["camera"]["params"])
    msgs = list(_messages(doc))
    for i, (uid, ids, corners) in enumerate(msgs):
        s.add_detections(uid, ids, corners)
        s.solve_incremental()
        for x in (o, alt):
            x.add_detections(uid, ids, corners)
            x.solve_incremental()
        _compare(s, o, alt, key=("cfg1_incremental", i), rms_rel=1e-8 if i == len(msgs) - 1 else None)
        if i == 0:   # the exemption's premise (spread_tol.EXEMPT): the flat-valley stop
            assert o.last_summary["termination"] == "NO_CONVERGENCE"
    assert s.num_solves == 3
    assert s.last_summary()["final_rms_px"] < 1.0
