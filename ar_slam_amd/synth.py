"""Seeded synthetic AR-tag bundle-adjustment graphs.

The reference has no fixtures on its hot path, so every
benchmark and parity graph is generated here from a fixed seed.  The model
is the reference's own:

* tag pose ``[t_t, w_t]`` maps tag-frame points to world,
  ``X_w = R(w_t) X_t + t_t`` (``ar_slam_util.cpp:144-148``); tags lie in the
  plane z = 0 with their z axis pointing away from the cameras (the marker
  faces the camera, as the reference's initialisers assume);
* capture ``inv_pose = [t_c, w_c]`` maps world to camera,
  ``X_c = R(w_c) (X_w + t_c)`` (``ar_slam_util.cpp:150-155``), so the
  camera centre is ``-t_c``;
* pinhole with focal only, centred pixel coordinates (``:157-162``);
* corners ``0.5 * aruco_size * ARUCO_DIRECTIONS[i]`` in TL, TR, BR, BL
  order (``ar_slam_util.hpp:319,340-345``).

Corner observations are the truth projected through that model plus
N(0, noise_px) pixel noise; the initial state is the truth perturbed by
N(0, 2 cm) on translations and N(0, 0.02 rad) on angle-axis components, and
the focal starts at 1.1 x truth.  Everything is numpy PCG64 seeded, so a
config name plus seed reproduces a graph bit for bit.
"""
from __future__ import annotations

import dataclasses

import numpy as np

IMG_W = 1020
IMG_H = 768
F_TRUE = 900.0
ARUCO_SIZE = 0.0635          # ar_slam_util.hpp:319
TAG_SPACING = 0.25
ARUCO_DIRECTIONS = np.array([[-1.0, -1.0], [1.0, -1.0], [1.0, 1.0], [-1.0, 1.0]])
DBL_EPS = np.finfo(np.float64).eps

# name -> (n_captures, grid_x, grid_y, seed).  cfg2/cfg3 are BASELINE.json
# configs[1]/[2]; the small ones are parity-test graphs.
CONFIGS = {
    "tiny": (6, 4, 3, 11),
    "small": (50, 6, 5, 12),
    "medium": (200, 10, 8, 13),
    "cfg2": (1000, 20, 15, 1),
    "cfg3": (10000, 50, 40, 2),
    # parity graph with SURVEY.md §8d's full rotation ranges: camera roll and
    # tag yaw ~ U(-pi, pi), so angle-axis vectors reach |w| ~ pi
    "wide": (300, 12, 10, 15),
    # BASELINE.json configs[0]: the demo's 3 images of 6 tags (resources/images
    # img1-3, demo_launch.py:39-110), replicated synthetically at 1020x768 --
    # detection needs OpenCV's ArUco dictionaries, absent from the image
    "cfg1": (3, 3, 2, 16),
    # parity graphs of larger captures (cameras 1.5-4 m from the tag plane):
    # 8, 11, 16, 40 and 64 tags per capture, capture 0 sees 80 ("kvar"); every
    # capture sees 24 ("k24"); a wall: 10 captures of 120 tags ("wall")
    "kvar": (60, 20, 15, 21),
    "k24": (80, 16, 12, 22),
    "wall": (10, 16, 12, 23),
}
FULL_ROTATION = {"wide"}
TAGS_PER_CAPTURE = {"cfg1": 4, "kvar": (80, 11, 16, 40, 64, 8, 8, 11, 16, 40, 64, 8), "k24": 24, "wall": 120}
DEPTH = {"kvar": (1.5, 4.0), "k24": (1.5, 3.0), "wall": (3.5, 4.5)}


@dataclasses.dataclass
class Graph:
    """Bundle-adjustment problem in SoA form (capture-major observations)."""

    camera: np.ndarray      # (3,)   f, l1, l2 (initial state)
    cap: np.ndarray         # (Nc,6) inv_pose t_c, w_c (initial state)
    tag: np.ndarray         # (Nt,6) pose t_t, w_t (initial state)
    obs_cap: np.ndarray     # (Nb,)  int32 capture index
    obs_tag: np.ndarray     # (Nb,)  int32 tag index
    corners: np.ndarray     # (Nb,8) observed x0,y0,...,x3,y3 (centred px)
    camera_true: np.ndarray
    cap_true: np.ndarray
    tag_true: np.ndarray
    name: str = ""

    @property
    def n_cap(self):
        return self.cap.shape[0]

    @property
    def n_tag(self):
        return self.tag.shape[0]

    @property
    def n_obs(self):
        return self.obs_cap.shape[0]

    def copy(self):
        return dataclasses.replace(
            self, camera=self.camera.copy(), cap=self.cap.copy(), tag=self.tag.copy())


def rodrigues(w):
    """Rotation matrices for angle-axis rows ``w`` (N,3) -> (N,3,3)."""
    w = np.atleast_2d(w)
    th = np.linalg.norm(w, axis=1)
    k = np.where(th[:, None] > 0, w / np.maximum(th, 1e-300)[:, None], 0.0)
    K = np.zeros((w.shape[0], 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -k[:, 2], k[:, 1]
    K[:, 1, 0], K[:, 1, 2] = k[:, 2], -k[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -k[:, 1], k[:, 0]
    s, c = np.sin(th)[:, None, None], np.cos(th)[:, None, None]
    return np.eye(3)[None] + s * K + (1 - c) * (K @ K)


def log_so3(R):
    """Angle-axis of rotation matrices (N,3,3) -> (N,3), valid up to pi."""
    R = np.asarray(R)
    tr = np.clip((np.trace(R, axis1=1, axis2=2) - 1.0) * 0.5, -1.0, 1.0)
    th = np.arccos(tr)
    v = np.stack([R[:, 2, 1] - R[:, 1, 2], R[:, 0, 2] - R[:, 2, 0], R[:, 1, 0] - R[:, 0, 1]], 1)
    out = np.zeros((R.shape[0], 3))
    small = th < 1e-6
    near_pi = th > np.pi - 1e-3
    reg = ~small & ~near_pi
    out[reg] = (th[reg] / (2 * np.sin(th[reg])))[:, None] * v[reg]
    out[small] = 0.5 * v[small]
    for i in np.nonzero(near_pi)[0]:
        # axis from the symmetric part: R = 2 k k^T - I at theta = pi
        B = (R[i] + np.eye(3)) * 0.5
        j = int(np.argmax(np.diag(B)))
        kk = B[:, j] / np.sqrt(max(B[j, j], 1e-300))
        kk /= np.linalg.norm(kk)
        if np.dot(kk, v[i]) < 0:
            kk = -kk
        out[i] = th[i] * kk
    return out


def angle_axis_rotate(w, x):
    """Vectorised restatement of ``ceres::AngleAxisRotatePoint`` (N,3),(N,3)."""
    w = np.atleast_2d(w)
    x = np.atleast_2d(x)
    th2 = np.sum(w * w, axis=1)
    big = th2 > DBL_EPS
    th = np.sqrt(np.where(big, th2, 1.0))
    c, s = np.cos(th), np.sin(th)
    u = w / th[:, None]
    cr = np.cross(u, x)
    tmp = np.sum(u * x, axis=1) * (1.0 - c)
    rot_big = x * c[:, None] + cr * s[:, None] + u * tmp[:, None]
    rot_small = x + np.cross(w, x)
    return np.where(big[:, None], rot_big, rot_small)


def project_corners(camera, cap, tag):
    """Project all 4 corners of each (cap row, tag row) pair -> (N,8)."""
    n = cap.shape[0]
    out = np.empty((n, 8))
    for i, d in enumerate(ARUCO_DIRECTIONS):
        corner = np.tile([0.5 * ARUCO_SIZE * d[0], 0.5 * ARUCO_SIZE * d[1], 0.0], (n, 1))
        a = angle_axis_rotate(tag[:, 3:], corner) + tag[:, :3]
        b = a + cap[:, :3]
        p = angle_axis_rotate(cap[:, 3:], b)
        out[:, 2 * i] = camera[0] * (p[:, 0] / p[:, 2])
        out[:, 2 * i + 1] = camera[0] * (p[:, 1] / p[:, 2])
    return out


def _rot_axis(axis, ang):
    return rodrigues(axis * ang[:, None])


def _sample_cameras(rng, n, x_lo, x_hi, y_lo, y_hi, max_tilt, roll_range=0.5 * np.pi, depth=(0.6, 1.2)):
    """World->camera rotations and centres of captures looking at the tag plane.

    World z points from the cameras towards the tag plane (z = 0), so an
    untilted camera has R = Rz(roll).  cfg2/cfg3 keep roll and tag yaw within
    +-90 deg (no pose near the angle-axis singularity at |w| = pi);
    roll_range = pi is SURVEY.md §8d's U(-pi, pi) (the "wide" parity graph).
    """
    pos = np.stack([rng.uniform(x_lo, x_hi, n), rng.uniform(y_lo, y_hi, n),
                    -rng.uniform(depth[0], depth[1], n)], 1)
    roll = rng.uniform(-roll_range, roll_range, n)
    tilt = rng.uniform(0.0, max_tilt, n)
    tilt_dir = rng.uniform(-np.pi, np.pi, n)
    R_roll = _rot_axis(np.tile([0, 0, 1.0], (n, 1)), roll)
    tilt_axis = np.stack([np.cos(tilt_dir), np.sin(tilt_dir), np.zeros(n)], 1)
    R_tilt = rodrigues(tilt_axis * tilt[:, None])
    R_wc = R_tilt @ R_roll
    R_cw = np.transpose(R_wc, (0, 2, 1))
    return R_cw, pos


def _visible_nearest(R_cw, pos, corners_w, centres, cand, k):
    """k nearest (3-D) fully visible tags among ``cand``; None if < k visible."""
    p = np.einsum("ij,tcj->tci", R_cw, corners_w[cand] - pos)
    z = p[..., 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        u = F_TRUE * p[..., 0] / z
        v = F_TRUE * p[..., 1] / z
    vis = ((z > 0.1) & (np.abs(u) < 0.5 * IMG_W - 1.0) & (np.abs(v) < 0.5 * IMG_H - 1.0)).all(1)
    if np.count_nonzero(vis) < k:
        return None
    d = np.linalg.norm(centres[cand] - pos, axis=1)
    d = np.where(vis, d, np.inf)
    order = np.lexsort((cand, d))          # ties broken by tag index
    return cand[order[:k]]


def make_graph(n_captures, grid_x, grid_y, seed, k=8, noise_px=0.5,
               init_trans_sigma=0.02, init_rot_sigma=0.02, f_init=1.1 * F_TRUE,
               max_tilt=np.deg2rad(20.0), name="", full_rotation=False, depth=(0.6, 1.2)):
    """Generate a connected capture/tag graph with exactly ``k`` tags per capture (``k`` an int,
    or a sequence: capture c sees ``k[c % len(k)]`` tags; cameras ``depth`` metres from the plane)."""
    ks = np.resize(np.asarray(k, np.int64), n_captures) if np.ndim(k) else np.full(n_captures, int(k))
    kmax = int(ks.max())
    rng = np.random.Generator(np.random.PCG64(seed))
    n_tag = grid_x * grid_y
    gx, gy = np.meshgrid(np.arange(grid_x) * TAG_SPACING, np.arange(grid_y) * TAG_SPACING)
    tag_true = np.zeros((n_tag, 6))
    tag_true[:, 0] = gx.ravel()
    tag_true[:, 1] = gy.ravel()
    # tags face the cameras: in the reference's marker frame (x right, y down,
    # z away from the viewer; ar_slam_util.hpp:340-345 and calcInitValues
    # :52-95) the tag z axis points away from the cameras, i.e. along world +z
    rot_range = np.pi if full_rotation else 0.5 * np.pi
    tag_true[:, 5] = rng.uniform(-rot_range, rot_range, n_tag)
    camera_true = np.array([F_TRUE, 0.0, 0.0])

    # tag corner world points (Nt,4,3)
    corners_w = np.empty((n_tag, 4, 3))
    for i, d in enumerate(ARUCO_DIRECTIONS):
        c = np.tile([0.5 * ARUCO_SIZE * d[0], 0.5 * ARUCO_SIZE * d[1], 0.0], (n_tag, 1))
        corners_w[:, i] = angle_axis_rotate(tag_true[:, 3:], c) + tag_true[:, :3]
    centres = tag_true[:, :3]

    x_lo, x_hi = -0.1, (grid_x - 1) * TAG_SPACING + 0.1
    y_lo, y_hi = -0.1, (grid_y - 1) * TAG_SPACING + 0.1
    cap_true = np.zeros((n_captures, 6))
    obs_tags = [None] * n_captures
    filled = 0
    n_cand = min(n_tag, max(128, 2 * kmax))
    while filled < n_captures:
        m = max(64, min(4096, (n_captures - filled) * 2))
        R_cw, pos = _sample_cameras(rng, m, x_lo, x_hi, y_lo, y_hi, max_tilt, rot_range, depth)
        # 3-D distance order == XY distance order (all tags at z = 0), so the
        # k nearest visible tags lie among the n_cand XY-nearest whenever at
        # least k of those are visible; otherwise fall back to every tag.
        d2 = ((centres[None, :, :2] - pos[:, None, :2]) ** 2).sum(-1)      # (m,Nt)
        cand = np.argpartition(d2, n_cand - 1, axis=1)[:, :n_cand] if n_cand < n_tag \
            else np.tile(np.arange(n_tag), (m, 1))
        for i in range(m):
            if filled >= n_captures:
                break
            sel = _visible_nearest(R_cw[i], pos[i], corners_w, centres, cand[i], ks[filled])
            if sel is None and n_cand < n_tag:
                sel = _visible_nearest(R_cw[i], pos[i], corners_w, centres, np.arange(n_tag), ks[filled])
            if sel is None:
                continue
            obs_tags[filled] = sel
            cap_true[filled, :3] = -pos[i]
            cap_true[filled, 3:] = log_so3(R_cw[i:i + 1])[0]
            filled += 1

    # connectivity (union-find over captures via shared tags)
    parent = np.arange(n_captures + n_tag)

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a
    for c in range(n_captures):
        for t in obs_tags[c]:
            ra, rb = find(c), find(n_captures + t)
            if ra != rb:
                parent[ra] = rb
    roots = {find(c) for c in range(n_captures)}
    if len(roots) != 1:
        raise RuntimeError(f"synthetic graph not connected ({len(roots)} components)")

    obs_cap = np.repeat(np.arange(n_captures), ks).astype(np.int32)
    obs_tag = np.concatenate(obs_tags).astype(np.int32)
    corners = project_corners(camera_true, cap_true[obs_cap], tag_true[obs_tag])
    corners += rng.normal(0.0, noise_px, corners.shape)

    cap0 = cap_true.copy()
    cap0[:, :3] += rng.normal(0.0, init_trans_sigma, (n_captures, 3))
    cap0[:, 3:] += rng.normal(0.0, init_rot_sigma, (n_captures, 3))
    tag0 = tag_true.copy()
    tag0[:, :3] += rng.normal(0.0, init_trans_sigma, (n_tag, 3))
    tag0[:, 3:] += rng.normal(0.0, init_rot_sigma, (n_tag, 3))
    camera0 = np.array([f_init, 0.0, 0.0])
    return Graph(camera0, cap0, tag0, obs_cap, obs_tag, np.ascontiguousarray(corners),
                 camera_true, cap_true, tag_true, name)


@dataclasses.dataclass
class LocalizeBatch:
    """Independent localize queries against a fixed map (cfg5).

    The map is a graph's tags at their true poses with the true focal, both
    constant (ar_slam_util.cpp:965,972); each query is one new capture whose
    observations ``[q_start[q], q_start[q+1])`` are in block order.
    """

    camera: np.ndarray      # (3,)
    tag: np.ndarray         # (Nt,6) map
    q_start: np.ndarray     # (Nq+1,) int32
    obs_tag: np.ndarray     # (Nb,) int32
    corners: np.ndarray     # (Nb,8)
    pose_true: np.ndarray   # (Nq,6)
    tag_in_map: np.ndarray  # (Nt,) uint8

    @property
    def n_query(self):
        return self.q_start.shape[0] - 1

    @property
    def n_obs(self):
        return self.obs_tag.shape[0]


def make_localize_batch(map_name="cfg3", n_query=4096, seed=3, k=8, noise_px=0.5,
                        max_tilt=np.deg2rad(20.0)):
    """cfg5: ``n_query`` captures of the ``map_name`` tag grid (truth), k tags each."""
    _, grid_x, grid_y, _ = CONFIGS[map_name]
    g = config_graph(map_name)
    tag = g.tag_true.copy()
    n_tag = tag.shape[0]
    rng = np.random.Generator(np.random.PCG64(seed))
    corners_w = np.empty((n_tag, 4, 3))
    for i, d in enumerate(ARUCO_DIRECTIONS):
        c = np.tile([0.5 * ARUCO_SIZE * d[0], 0.5 * ARUCO_SIZE * d[1], 0.0], (n_tag, 1))
        corners_w[:, i] = angle_axis_rotate(tag[:, 3:], c) + tag[:, :3]
    centres = tag[:, :3]
    x_lo, x_hi = -0.1, (grid_x - 1) * TAG_SPACING + 0.1
    y_lo, y_hi = -0.1, (grid_y - 1) * TAG_SPACING + 0.1
    pose = np.zeros((n_query, 6))
    obs = np.zeros((n_query, k), np.int64)
    filled = 0
    n_cand = min(n_tag, 128)
    while filled < n_query:
        m = max(64, min(4096, (n_query - filled) * 2))
        R_cw, pos = _sample_cameras(rng, m, x_lo, x_hi, y_lo, y_hi, max_tilt)
        d2 = ((centres[None, :, :2] - pos[:, None, :2]) ** 2).sum(-1)
        cand = np.argpartition(d2, n_cand - 1, axis=1)[:, :n_cand] if n_cand < n_tag \
            else np.tile(np.arange(n_tag), (m, 1))
        for i in range(m):
            if filled >= n_query:
                break
            sel = _visible_nearest(R_cw[i], pos[i], corners_w, centres, cand[i], k)
            if sel is None:
                continue
            obs[filled] = sel
            pose[filled, :3] = -pos[i]
            pose[filled, 3:] = log_so3(R_cw[i:i + 1])[0]
            filled += 1
    q_of = np.repeat(np.arange(n_query), k)
    obs_tag = obs.ravel().astype(np.int32)
    corners = project_corners(g.camera_true, pose[q_of], tag[obs_tag])
    corners += rng.normal(0.0, noise_px, corners.shape)
    return LocalizeBatch(g.camera_true.copy(), tag, (np.arange(n_query + 1) * k).astype(np.int32),
                         obs_tag, np.ascontiguousarray(corners), pose, np.ones(n_tag, np.uint8))


def config_graph(name, **kw):
    n, gx, gy, seed = CONFIGS[name]
    if name in FULL_ROTATION:
        kw.setdefault("full_rotation", True)
    if name in TAGS_PER_CAPTURE:
        kw.setdefault("k", TAGS_PER_CAPTURE[name])
    if name in DEPTH:
        kw.setdefault("depth", DEPTH[name])
    return make_graph(n, gx, gy, seed, name=name, **kw)


def rms_px(cost, n_obs):
    """Reprojection RMS per corner, sqrt(2 cost / (4 N_obs))."""
    return float(np.sqrt(2.0 * cost / (4.0 * n_obs))) if n_obs else 0.0


def prefix_graph(g, k):
    """The first k captures of g and the tags they see (renumbered in first-seen index order):
    the problem ArSlamSolver::solveIncremental solves after its k-th capture
    (ar_slam_util.cpp:629-742, one Solve of the whole problem so far)."""
    sel = g.obs_cap < k
    tags, inv = np.unique(g.obs_tag[sel], return_inverse=True)
    return Graph(camera=g.camera.copy(), cap=g.cap[:k].copy(), tag=g.tag[tags].copy(),
                 obs_cap=g.obs_cap[sel].astype(np.int32), obs_tag=inv.astype(np.int32),
                 corners=g.corners[sel], camera_true=g.camera_true, cap_true=g.cap_true[:k],
                 tag_true=g.tag_true[tags], name=f"{g.name}[:{k}]")

