"""ctypes binding of the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See
arslam_oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

MAX_ITERS = 1024
ELIM_CAPTURES, ELIM_NONE, ELIM_MIXED = 0, 1, 2   # or_options.elimination
TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}
RULES = {0: "none", 1: "gradient_tolerance", 2: "parameter_tolerance", 3: "function_tolerance",
         4: "min_trust_region_radius", 5: "max_num_iterations", 6: "invalid_steps",
         7: "evaluation_failed"}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_up = C.POINTER(C.c_ubyte)


class Problem(C.Structure):
    _fields_ = [("n_cap", C.c_int), ("n_tag", C.c_int), ("n_obs", C.c_int),
                ("camera", _dp), ("cap", _dp), ("tag", _dp),
                ("obs_cap", _ip), ("obs_tag", _ip), ("corners", _dp),
                ("camera_const", C.c_int), ("cap_const", _up), ("tag_const", _up)]


class Options(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int),
                ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double),
                ("initial_trust_region_radius", C.c_double),
                ("max_trust_region_radius", C.c_double),
                ("min_trust_region_radius", C.c_double),
                ("min_relative_decrease", C.c_double),
                ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
                ("max_num_consecutive_invalid_steps", C.c_int),
                ("jacobi_scaling", C.c_int), ("elimination", C.c_int),
                ("num_threads", C.c_int), ("progress", C.c_int),
                ("debug_indefinite_mask", C.c_ulonglong),
                ("e_cap", _up), ("e_tag", _up)]


class Iter(C.Structure):
    _fields_ = [("iteration", C.c_int),
                ("cost", C.c_double), ("cost_change", C.c_double),
                ("gradient_max_norm", C.c_double), ("gradient_norm", C.c_double),
                ("step_norm", C.c_double), ("relative_decrease", C.c_double),
                ("trust_region_radius", C.c_double),
                ("step_is_valid", C.c_int), ("step_is_successful", C.c_int),
                ("iteration_time", C.c_double), ("cumulative_time", C.c_double)]


class Summary(C.Structure):
    _fields_ = [("termination", C.c_int), ("rule", C.c_int),
                ("num_successful_steps", C.c_int), ("num_unsuccessful_steps", C.c_int),
                ("num_linear_solves", C.c_int),
                ("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("fixed_cost", C.c_double), ("n_iters", C.c_int),
                ("iters", Iter * (MAX_ITERS + 1))]


class Comm(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("rank", C.c_int),
                ("allreduce_sum", C.CFUNCTYPE(None, C.c_void_p, _dp, C.c_long)),
                ("allreduce_max", C.CFUNCTYPE(None, C.c_void_p, _dp, C.c_long))]


_REDUCE_T = C.CFUNCTYPE(None, C.c_void_p, _dp, C.c_long)
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_default_options.argtypes = [C.POINTER(Options)]
        L.or_angle_axis_rotate.argtypes = [_dp, _dp, _dp]
        L.or_residual.argtypes = [_dp, _dp, _dp, _dp, _dp]
        L.or_residual_jacobian.argtypes = [_dp, _dp, _dp, _dp, _dp, _dp]
        L.or_cost.argtypes = [C.POINTER(Problem)]
        L.or_cost.restype = C.c_double
        L.or_solve.argtypes = [C.POINTER(Problem), C.POINTER(Options), C.POINTER(Summary),
                               C.POINTER(Comm)]
        L.or_solve.restype = C.c_int
        L.or_llt_lower.argtypes = [_dp, C.c_long, C.c_long, C.c_int]
        L.or_llt_lower.restype = C.c_int
        L.or_init_capture_pose.argtypes = [_dp, _dp, _dp, _dp]
        L.or_init_ar_pose.argtypes = [_dp, _dp, _dp, _dp]
        L.or_compose_axis_angle.argtypes = [_dp, _dp, _dp]
        L.or_calc_init_values.argtypes = [_dp, C.c_double, _dp]
        L.or_localize_many.argtypes = [C.c_int, _ip, _ip, _dp, _dp, _dp, C.c_int, C.POINTER(C.c_ubyte),
                                       C.c_int, _dp, C.POINTER(Options), _ip, C.POINTER(Summary)]
        L.or_localize_many.restype = C.c_int
        _lib = L
    return _lib


def _p(a, t=_dp):
    return a.ctypes.data_as(t)


def default_options(**kw):
    o = Options()
    lib().or_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def residual_jacobian(cam, cap, tag, corners):
    cam, cap, tag, corners = (np.ascontiguousarray(a, np.float64) for a in (cam, cap, tag, corners))
    r = np.zeros(8)
    J = np.zeros((8, 15))
    lib().or_residual_jacobian(_p(cam), _p(cap), _p(tag), _p(corners), _p(r), _p(J))
    return r, J


def residual(cam, cap, tag, corners):
    cam, cap, tag, corners = (np.ascontiguousarray(a, np.float64) for a in (cam, cap, tag, corners))
    r = np.zeros(8)
    lib().or_residual(_p(cam), _p(cap), _p(tag), _p(corners), _p(r))
    return r


def llt_lower(A, num_threads=1):
    """In-place lower Cholesky of a C-contiguous float64 square matrix."""
    n = A.shape[0]
    return lib().or_llt_lower(_p(A), n, A.shape[1], num_threads)


class _Arrays:
    """Keeps numpy buffers alive behind a Problem struct."""

    def __init__(self, camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False,
                 cap_const=None, tag_const=None):
        self.camera = np.ascontiguousarray(camera, np.float64).copy()
        self.cap = np.ascontiguousarray(cap, np.float64).reshape(-1, 6).copy()
        self.tag = np.ascontiguousarray(tag, np.float64).reshape(-1, 6).copy()
        self.obs_cap = np.ascontiguousarray(obs_cap, np.int32)
        self.obs_tag = np.ascontiguousarray(obs_tag, np.int32)
        self.corners = np.ascontiguousarray(corners, np.float64).reshape(-1, 8)
        self.cap_const = None if cap_const is None else np.ascontiguousarray(cap_const, np.uint8)
        self.tag_const = None if tag_const is None else np.ascontiguousarray(tag_const, np.uint8)
        self.prob = Problem(self.cap.shape[0], self.tag.shape[0], self.obs_cap.shape[0],
                            _p(self.camera), _p(self.cap), _p(self.tag),
                            _p(self.obs_cap, _ip), _p(self.obs_tag, _ip), _p(self.corners),
                            int(bool(camera_const)),
                            None if self.cap_const is None else _p(self.cap_const, _up),
                            None if self.tag_const is None else _p(self.tag_const, _up))


def summary_dict(s):
    its = [{f: getattr(s.iters[i], f) for f, _ in Iter._fields_} for i in range(s.n_iters)]
    return {"termination": TERMINATION[s.termination], "rule": RULES[s.rule],
            "num_successful_steps": s.num_successful_steps,
            "num_unsuccessful_steps": s.num_unsuccessful_steps,
            "num_linear_solves": s.num_linear_solves,
            "initial_cost": s.initial_cost, "final_cost": s.final_cost,
            "fixed_cost": s.fixed_cost, "iterations": its}


def solve(camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False, cap_const=None,
          tag_const=None, comm=None, **opts):
    """Run the oracle LM; returns (camera, cap, tag, summary_dict)."""
    A = _Arrays(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
    # (elimination=ELIM_MIXED: e_cap / e_tag are the eliminated captures and tags, kept alive here)
    keep = {k: np.ascontiguousarray(opts.pop(k), np.uint8) for k in ("e_cap", "e_tag") if k in opts}
    o = default_options(**opts)
    for k, v in keep.items():
        setattr(o, k, _p(v, _up))
    s = Summary()
    lib().or_solve(C.byref(A.prob), C.byref(o), C.byref(s), None if comm is None else C.byref(comm))
    return A.camera, A.cap, A.tag, summary_dict(s)


def solve_graph(g, **opts):
    return solve(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, **opts)


def init_capture_pose(corners, camera, ar_pose):
    """initCapturePose (ar_slam_util.cpp:98-115) -> inv_cap_pose (6,)."""
    c, cam, ar = (np.ascontiguousarray(a, np.float64) for a in (corners, camera, ar_pose))
    out = np.zeros(6)
    lib().or_init_capture_pose(_p(c), _p(cam), _p(ar), _p(out))
    return out


def init_ar_pose(corners, camera, inv_cap_pose):
    """initArPose (ar_slam_util.cpp:118-128) -> ar_pose (6,)."""
    c, cam, cp = (np.ascontiguousarray(a, np.float64) for a in (corners, camera, inv_cap_pose))
    out = np.zeros(6)
    lib().or_init_ar_pose(_p(c), _p(cam), _p(cp), _p(out))
    return out


def compose_axis_angle(r1, r2):
    a, b = (np.ascontiguousarray(x, np.float64) for x in (r1, r2))
    out = np.zeros(3)
    lib().or_compose_axis_angle(_p(a), _p(b), _p(out))
    return out


def localize_many(batch, init_from_map=True, pose=None, with_summaries=False, **opts):
    """localizeMany (ar_slam_util.cpp:888-979) over a synth.LocalizeBatch.

    Returns (pose (Nq,6), status (Nq,) with -1 for skipped queries, summaries or None)."""
    nq = batch.n_query
    pose = np.zeros((nq, 6)) if pose is None else np.ascontiguousarray(pose, np.float64).copy()
    status = np.zeros(nq, np.int32)
    q_start = np.ascontiguousarray(batch.q_start, np.int32)
    obs_tag = np.ascontiguousarray(batch.obs_tag, np.int32)
    corners = np.ascontiguousarray(batch.corners, np.float64)
    camera = np.ascontiguousarray(batch.camera, np.float64)
    tag = np.ascontiguousarray(batch.tag, np.float64)
    tim = None if batch.tag_in_map is None else np.ascontiguousarray(batch.tag_in_map, np.uint8)
    sums = (Summary * nq)() if with_summaries else None
    o = default_options(**opts)
    lib().or_localize_many(nq, _p(q_start, _ip), _p(obs_tag, _ip), _p(corners), _p(camera), _p(tag),
                           tag.shape[0], None if tim is None else tim.ctypes.data_as(C.POINTER(C.c_ubyte)),
                           int(bool(init_from_map)), _p(pose), C.byref(o), _p(status, _ip), sums)
    return pose, status, ([summary_dict(s) for s in sums] if with_summaries else None)


def make_comm(rank, sum_fn, max_fn):
    """Build an or_comm from two python callables f(np.ndarray) -> None (in place)."""

    def _wrap(fn):
        def cb(ctx, ptr, n):
            if n <= 0:
                return
            arr = np.ctypeslib.as_array(ptr, shape=(n,))
            fn(arr)
        return _REDUCE_T(cb)
    cs, cm = _wrap(sum_fn), _wrap(max_fn)
    comm = Comm(None, rank, cs, cm)
    comm._keep = (cs, cm)
    return comm


def cost(camera, cap, tag, obs_cap, obs_tag, corners):
    A = _Arrays(camera, cap, tag, obs_cap, obs_tag, corners)
    return lib().or_cost(C.byref(A.prob))
