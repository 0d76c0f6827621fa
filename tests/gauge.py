"""Gauge-aligned comparison of two solved maps (test helper, no GPU).

The mapping problem has a 6-DoF gauge freedom (no block is held constant in
the reference's solve, ar_slam_util.cpp:1001-1018), so two solvers that sum in
different orders may end a rounding-level rigid motion apart.  One rigid
motion G (x -> R x + t) is fitted on the tag positions (Kabsch) and applied to
every pose of one solution before it is compared with the other:

* tag pose [t_t, w_t] maps tag points to world (ar_slam_util.cpp:144-148):
  t_t -> R t_t + t,  R(w_t) -> R R(w_t);
* capture inv_pose [t_c, w_c] maps world to camera, X_c = R(w_c)(X_w + t_c)
  (:150-155), so its centre -t_c -> R(-t_c) + t and R(w_c) -> R(w_c) R^T.

Rotation differences are the angle of R_a^T R_b, computed as
2 asin(|R_a - R_b|_F / (2 sqrt 2)) (exact to rounding at small angles).
"""
import json
import os

import numpy as np

from ar_slam_amd.synth import rodrigues


def fit_rigid(P, Q):
    """(R, t) minimising |R P + t - Q| over rows (Kabsch, proper rotation)."""
    pc, qc = P.mean(0), Q.mean(0)
    U, _, Vt = np.linalg.svd((P - pc).T @ (Q - qc))
    d = np.sign(np.linalg.det(Vt.T @ U.T))
    R = Vt.T @ np.diag([1, 1, d]) @ U.T
    return R, qc - R @ pc


def align_rigid(P, Q):
    """P's rows rigidly aligned onto Q's."""
    R, t = fit_rigid(P, Q)
    return P @ R.T + t


def rot_angle(Ra, Rb):
    """Angle (rad) between stacks of rotation matrices."""
    f = np.linalg.norm((Ra - Rb).reshape(len(Ra), -1), axis=1)
    return 2.0 * np.arcsin(np.minimum(f / (2.0 * np.sqrt(2.0)), 1.0))


def pose_errors(cap_o, tag_o, cap_r, tag_r, tags=None, caps=None):
    """Max position (m) and rotation (rad) errors of the captures and tags of solution o, moved
    into solution r's gauge by the rigid motion fitted on the tag positions.  Returns a dict."""
    tags = np.arange(len(tag_r)) if tags is None else np.asarray(tags)
    caps = np.arange(len(cap_r)) if caps is None else np.asarray(caps)
    R, t = fit_rigid(tag_o[tags, :3], tag_r[tags, :3])
    out = {}
    tp = tag_o[tags, :3] @ R.T + t
    out["tag_pos"] = float(np.abs(tp - tag_r[tags, :3]).max()) if len(tags) else 0.0
    out["tag_rot"] = float(rot_angle(R[None] @ rodrigues(tag_o[tags, 3:]), rodrigues(tag_r[tags, 3:])).max()) \
        if len(tags) else 0.0
    if len(caps):
        cc = (-cap_o[caps, :3]) @ R.T + t
        out["cap_pos"] = float(np.abs(cc - (-cap_r[caps, :3])).max())
        out["cap_rot"] = float(rot_angle(rodrigues(cap_o[caps, 3:]) @ R.T[None], rodrigues(cap_r[caps, 3:])).max())
    else:
        out["cap_pos"] = out["cap_rot"] = 0.0
    return out


# VERDICT r03 "next round" item 1: positions 1e-6 m, rotations 1e-7 rad
POS_TOL = 1e-6
ROT_TOL = 1e-7


def assert_poses_match(cap_o, tag_o, cap_r, tag_r, tags=None, caps=None, pos_tol=POS_TOL, rot_tol=ROT_TOL):
    e = pose_errors(cap_o, tag_o, cap_r, tag_r, tags, caps)
    assert e["tag_pos"] < pos_tol and e["cap_pos"] < pos_tol, e
    assert e["tag_rot"] < rot_tol and e["cap_rot"] < rot_tol, e
    return e


def load_cfg3_golden():
    """tests/golden/lm_cfg3.json (the trace) and lm_cfg3_final.npz (the oracle's final camera,
    10k capture and 2k tag poses), made by make_golden.py; the oracle takes minutes here."""
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(d, "lm_cfg3.json")) as f:
        gold = json.load(f)
    with np.load(os.path.join(d, "lm_cfg3_final.npz")) as z:
        final = {k: z[k] for k in z.files}
    return gold, final
