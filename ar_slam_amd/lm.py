"""Python binding of libarslam_lm.so (ctypes over the C-ABI in include/arslam_lm.h).

This is the host-side mirror of the reference's solver interface used by the
tests, the benchmark and smoke():

* :class:`Problem` mirrors ``ceres::Problem`` as ArSlamSolver drives it --
  ``add_residual_block(corners, camera, capture, tag)`` is
  ``AddResidualBlock(AutoDiff<ArucoReprojectionError,8,3,6,6>, nullptr,
  camera, capture, aruco)`` (ar_slam_util.cpp:720-727),
  ``set_parameter_block_constant`` is ``SetParameterBlockConstant``
  (:965, :972) and ``solve`` is ``ceres::Solve`` (:1015); parameter blocks
  are caller-owned float64 numpy arrays updated in place.
* :func:`solve_soa` / :class:`ResidentProblem` are the bulk struct-of-arrays
  path (problem uploaded once to HBM, solved many times).

There is no CPU fallback: if the HIP library is missing or no GPU is
present, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ARSLAM_LIB") or os.path.join(HERE, "libarslam_lm.so")   # (override: variant builds)
MAX_ITERS = 1024
COMM_ID_BYTES = 128

TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE", 3: "USER_SUCCESS", 4: "USER_FAILURE"}
RULES = {0: "none", 1: "gradient_tolerance", 2: "parameter_tolerance", 3: "function_tolerance",
         4: "min_trust_region_radius", 5: "max_num_iterations", 6: "invalid_steps",
         7: "evaluation_failed", 8: "user_callback"}
ERRORS = {-1: "INVALID_ARG", -2: "UNSUPPORTED", -3: "NO_DEVICE", -4: "HIP", -5: "OUT_OF_MEMORY",
          -6: "COMM", -7: "STATE", -8: "DEVICE"}

# Every symbol include/arslam_lm.h declares (checked by the CPU tests).
EXPORTS = ["arslam_lm_options_init", "arslam_lm_create", "arslam_lm_destroy",
           "arslam_lm_set_options", "arslam_lm_get_options",
           "arslam_lm_add_residual_block", "arslam_lm_set_parameter_block_constant",
           "arslam_lm_set_parameter_block_variable", "arslam_lm_solve", "arslam_lm_reset",
           "arslam_lm_num_residual_blocks", "arslam_lm_load_soa", "arslam_lm_solve_loaded",
           "arslam_lm_solve_soa", "arslam_comm_unique_id", "arslam_lm_set_comm", "arslam_lm_set_comm_callback",
           "arslam_device_count", "arslam_lm_last_error", "arslam_lm_version",
           "arslam_lm_set_iteration_callback", "arslam_lm_owned_captures",
           "arslam_debug_residual_jacobian", "arslam_debug_dense_llt", "arslam_debug_dense_llt_ex",
           "arslam_debug_angle_axis_rotate", "arslam_lm_debug_force_indefinite",
           "arslam_lm_debug_force_multirank", "arslam_lm_debug_break_dependency", "arslam_lm_debug_tag_pair_tile",
           "arslam_debug_reduced_plan", "arslam_debug_reduced_plan_side", "arslam_debug_schur_stamps", "arslam_debug_ceres_e_blocks",
           "arslam_debug_mixed_groups",
           "arslam_debug_dag_simulate", "arslam_debug_dag_simulate_started", "arslam_debug_dag_workgroup_limit",
           "arslam_debug_dag_fault_detail", "arslam_debug_box_fingerprint",
           "arslam_debug_rank_split", "arslam_debug_gather_extend",
           "arslam_localize_many", "arslam_localizer_create", "arslam_localizer_destroy",
           "arslam_localizer_load", "arslam_localizer_solve",
           "arslam_slam_create", "arslam_slam_destroy", "arslam_slam_set_verbose", "arslam_slam_load_yaml",
           "arslam_slam_load_yaml_string", "arslam_slam_save_yaml", "arslam_slam_add_detections",
           "arslam_slam_solve", "arslam_slam_solve_incremental", "arslam_slam_localize_many",
           "arslam_slam_num_captures", "arslam_slam_num_arucos", "arslam_slam_num_blocks",
           "arslam_slam_num_solves", "arslam_slam_last_summary", "arslam_slam_solve_summary",
           "arslam_slam_solve_capture", "arslam_slam_unsolved_captures", "arslam_slam_capture", "arslam_slam_set_capture_pose", "arslam_slam_aruco", "arslam_slam_set_aruco_pose",
           "arslam_slam_block", "arslam_slam_camera", "arslam_slam_set_camera",
           "arslam_slam_get_transforms", "arslam_slam_camera_info"]

_dp = C.POINTER(C.c_double)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int)
SOLVER_CONTINUE, SOLVER_ABORT, SOLVER_TERMINATE_SUCCESSFULLY = 0, 1, 2
ELIM_AUTO, ELIM_CAPTURES, ELIM_TAGS, ELIM_MIXED = 0, 1, 2, 3   # arslam_lm_options.elimination
SETUP_LOAD, SETUP_VALUES, SETUP_APPEND = 0, 1, 2   # arslam_lm_summary.setup_kind
_ip = C.POINTER(C.c_int)
_up = C.POINTER(C.c_ubyte)


class LMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"arslam_lm error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


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
                ("minimizer_progress_to_stdout", C.c_int),
                ("update_state_every_iteration", C.c_int),
                ("device", C.c_int), ("cholesky_skip_zero_tiles", C.c_int),
                ("reduced_ordering", C.c_int), ("kernel_timing", C.c_int), ("factor_executor", C.c_int),
                ("phase_timing", C.c_int)]


class Iteration(C.Structure):
    _fields_ = [("iteration", C.c_int),
                ("cost", C.c_double), ("cost_change", C.c_double),
                ("gradient_max_norm", C.c_double), ("gradient_norm", C.c_double),
                ("step_norm", C.c_double), ("relative_decrease", C.c_double),
                ("trust_region_radius", C.c_double),
                ("step_is_valid", C.c_int), ("step_is_successful", C.c_int),
                ("iteration_time", C.c_double), ("cumulative_time", C.c_double)]


ITER_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(Iteration))


class Summary(C.Structure):
    _fields_ = [("termination", C.c_int), ("rule", C.c_int),
                ("num_successful_steps", C.c_int), ("num_unsuccessful_steps", C.c_int),
                ("num_linear_solves", C.c_int),
                ("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("fixed_cost", C.c_double), ("final_rms_px", C.c_double),
                ("n_obs", C.c_int), ("n_reduced", C.c_int),
                ("setup_time_s", C.c_double), ("setup_kind", C.c_int), ("minimizer_time_s", C.c_double),
                ("total_time_s", C.c_double),
                ("t_linearize_ms", C.c_double), ("t_schur_ms", C.c_double),
                ("t_cholesky_ms", C.c_double), ("t_solve_ms", C.c_double),
                ("t_backsub_ms", C.c_double), ("t_cost_ms", C.c_double),
                ("t_dominant_ms", C.c_double), ("dominant_flops", C.c_double),
                ("n_dominant_launches", C.c_long),
                ("n_factor_tiles", C.c_long), ("n_levels", C.c_int), ("n_update_tiles", C.c_long),
                ("factor_update_flops", C.c_double), ("factor_scalar_flops", C.c_double),
                ("comm_bytes", C.c_double),
                ("elimination_used", C.c_int), ("ceres_e_captures", C.c_int), ("ceres_e_tags", C.c_int),
                ("n_ranks", C.c_int), ("n_owned_captures", C.c_int), ("n_top_tiles", C.c_long),
                ("split_top_work", C.c_double), ("split_max_rank_work", C.c_double),
                ("split_total_work", C.c_double), ("t_factor_own_ms", C.c_double),
                ("t_factor_top_ms", C.c_double),
                ("n_iters", C.c_int), ("iters", Iteration * (MAX_ITERS + 1)),
                ("setup_phase_s", C.c_double * 5), ("comm_calls", C.c_long), ("n_active_ranks", C.c_int),
                ("order_reused", C.c_int)]

    def to_dict(self):
        its = [{f: getattr(self.iters[i], f) for f, _ in Iteration._fields_}
               for i in range(self.n_iters)]
        d = {f: getattr(self, f) for f, _ in Summary._fields_ if f not in ("iters", "termination", "rule")}
        d["setup_phase_s"] = list(self.setup_phase_s)
        d["termination"] = TERMINATION[self.termination]
        d["rule"] = RULES[self.rule]
        d["iterations"] = its
        return d


class SoaProblem(C.Structure):
    _fields_ = [("n_cap", C.c_int), ("n_tag", C.c_int), ("n_obs", C.c_int),
                ("camera", _dp), ("cap", _dp), ("tag", _dp),
                ("obs_cap", _ip), ("obs_tag", _ip), ("corners", _dp),
                ("camera_const", C.c_int), ("cap_const", _up), ("tag_const", _up)]


_lib = None


def library_path():
    return LIB_PATH


def library_info():
    """Which library this process measures: its file, the sha256 of the file (first 12 hex) and the
    build it reports (commit + source digest, ar_slam_amd/build.py build_id)."""
    import hashlib
    with open(LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:12]
    v = lib().arslam_lm_version().decode()
    return {"file": os.path.basename(LIB_PATH), "sha256": sha, "version": v.split(" build ")[0],
            "build": v.split(" build ")[-1] if " build " in v else "unknown"}


def lib():
    """Load the HIP library (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -m ar_slam_amd.build` "
                          "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    L.arslam_lm_options_init.argtypes = [C.POINTER(Options)]
    L.arslam_lm_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(Options)]
    L.arslam_lm_set_comm_callback.argtypes = [C.c_void_p, C.c_int, C.c_int, ALLREDUCE_FN, C.c_void_p]
    L.arslam_lm_set_options.argtypes = [C.c_void_p, C.POINTER(Options)]
    L.arslam_debug_rank_split.argtypes = [C.POINTER(SoaProblem), C.c_int, C.c_int, C.POINTER(SplitInfo), _ip]
    L.arslam_lm_owned_captures.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int)]
    for fn in ("arslam_slam_destroy", "arslam_slam_set_verbose", "arslam_slam_load_yaml",
               "arslam_slam_load_yaml_string", "arslam_slam_save_yaml", "arslam_slam_add_detections",
               "arslam_slam_solve", "arslam_slam_solve_incremental", "arslam_slam_localize_many",
               "arslam_slam_num_captures", "arslam_slam_num_arucos", "arslam_slam_num_blocks",
               "arslam_slam_num_solves", "arslam_slam_last_summary", "arslam_slam_solve_summary",
               "arslam_slam_solve_capture", "arslam_slam_unsolved_captures", "arslam_slam_capture",
               "arslam_slam_set_capture_pose", "arslam_slam_aruco", "arslam_slam_set_aruco_pose",
               "arslam_slam_block", "arslam_slam_camera", "arslam_slam_set_camera",
               "arslam_slam_get_transforms", "arslam_slam_camera_info"):
        getattr(L, fn).argtypes = None
    L.arslam_slam_destroy.restype = None
    L.arslam_slam_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(Options)]
    L.arslam_localize_many.argtypes = [C.POINTER(LocalizeBatchC), C.POINTER(Options), C.POINTER(LocalizeResult)]
    L.arslam_localizer_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(Options)]
    L.arslam_localizer_destroy.argtypes = [C.c_void_p]
    L.arslam_localizer_destroy.restype = None
    L.arslam_localizer_load.argtypes = [C.c_void_p, C.POINTER(LocalizeBatchC)]
    L.arslam_localizer_solve.argtypes = [C.c_void_p, _dp, C.POINTER(LocalizeResult), C.POINTER(C.c_double)]
    L.arslam_lm_get_options.argtypes = [C.c_void_p, C.POINTER(Options)]
    L.arslam_lm_destroy.argtypes = [C.c_void_p]
    L.arslam_lm_destroy.restype = None
    L.arslam_lm_add_residual_block.argtypes = [C.c_void_p, _dp, _dp, _dp, _dp]
    L.arslam_lm_set_parameter_block_constant.argtypes = [C.c_void_p, _dp]
    L.arslam_lm_set_parameter_block_variable.argtypes = [C.c_void_p, _dp]
    L.arslam_lm_solve.argtypes = [C.c_void_p, C.POINTER(Summary)]
    L.arslam_lm_reset.argtypes = [C.c_void_p]
    L.arslam_lm_num_residual_blocks.argtypes = [C.c_void_p]
    L.arslam_lm_load_soa.argtypes = [C.c_void_p, C.POINTER(SoaProblem)]
    L.arslam_lm_solve_loaded.argtypes = [C.c_void_p, C.POINTER(Summary)]
    L.arslam_lm_solve_soa.argtypes = [C.POINTER(SoaProblem), C.POINTER(Options), C.POINTER(Summary)]
    L.arslam_comm_unique_id.argtypes = [C.c_char_p]
    L.arslam_lm_set_comm.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p]
    L.arslam_device_count.argtypes = []
    L.arslam_lm_last_error.restype = C.c_char_p
    L.arslam_lm_version.restype = C.c_char_p
    L.arslam_debug_residual_jacobian.argtypes = [C.c_int, _dp, _dp, _dp, _dp, _dp, _dp]
    L.arslam_debug_dense_llt.argtypes = [C.c_long, _dp, _dp, _dp, C.POINTER(C.c_int)]
    L.arslam_debug_angle_axis_rotate.argtypes = [C.c_int, _dp, _dp, _dp, _ip]
    L.arslam_debug_ceres_e_blocks.argtypes = [C.POINTER(SoaProblem), _ip]
    L.arslam_debug_mixed_groups.argtypes = [C.POINTER(SoaProblem), _ip, C.POINTER(C.c_ubyte), C.POINTER(C.c_ubyte)]
    L.arslam_lm_debug_force_indefinite.argtypes = [C.c_void_p, C.c_ulonglong]
    L.arslam_lm_debug_force_multirank.argtypes = [C.c_void_p, C.c_int]
    L.arslam_debug_dag_workgroup_limit.argtypes = [C.c_int]
    L.arslam_lm_set_iteration_callback.argtypes = [C.c_void_p, ITER_CB, C.c_void_p]
    L.arslam_lm_debug_break_dependency.argtypes = [C.c_void_p, C.c_long, C.POINTER(C.c_long)]
    if hasattr(L, "arslam_lm_debug_tag_pair_tile"):   # (absent from older variant builds under A/B)
        L.arslam_lm_debug_tag_pair_tile.argtypes = [C.c_void_p, _dp, _dp, C.POINTER(C.c_int)]
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise LMError(rc, lib().arslam_lm_last_error().decode(errors="replace"))


def device_count():
    return lib().arslam_device_count()


def make_options(**kw):
    o = Options()
    lib().arslam_lm_options_init(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(f"unknown solver option {k}")
        setattr(o, k, v)
    return o


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


class _Soa:
    def __init__(self, camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False,
                 cap_const=None, tag_const=None):
        self.camera = _f64(camera).copy()
        self.cap = _f64(cap, (-1, 6)).copy()
        self.tag = _f64(tag, (-1, 6)).copy()
        self.obs_cap = np.ascontiguousarray(obs_cap, np.int32)
        self.obs_tag = np.ascontiguousarray(obs_tag, np.int32)
        self.corners = _f64(corners, (-1, 8))
        self.cap_const = None if cap_const is None else np.ascontiguousarray(cap_const, np.uint8)
        self.tag_const = None if tag_const is None else np.ascontiguousarray(tag_const, np.uint8)
        self.s = SoaProblem(self.cap.shape[0], self.tag.shape[0], self.obs_cap.shape[0],
                            self.camera.ctypes.data_as(_dp), self.cap.ctypes.data_as(_dp),
                            self.tag.ctypes.data_as(_dp), self.obs_cap.ctypes.data_as(_ip),
                            self.obs_tag.ctypes.data_as(_ip), self.corners.ctypes.data_as(_dp),
                            int(bool(camera_const)),
                            None if self.cap_const is None else self.cap_const.ctypes.data_as(_up),
                            None if self.tag_const is None else self.tag_const.ctypes.data_as(_up))


def solve_soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False, cap_const=None,
              tag_const=None, **opts):
    """One-shot bulk solve.  Returns (camera, cap, tag, summary dict)."""
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
    s = Summary()
    _check(lib().arslam_lm_solve_soa(C.byref(A.s), C.byref(make_options(**opts)), C.byref(s)))
    return A.camera, A.cap, A.tag, s.to_dict()


def warm_up(device=0):
    """One small solve (the 'tiny' synthetic graph) on `device`: the process's one-time runtime
    start (the library's code objects loaded on first launch, its stream, page-locked buffers),
    which a first load would otherwise carry.  Returns its wall time (s)."""
    import time
    from . import synth
    t = time.perf_counter()
    g = synth.config_graph("tiny")
    ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, device=device).solve()
    return time.perf_counter() - t


def solve_graph(g, **opts):
    return solve_soa(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, **opts)


class _Handle:
    def __init__(self, **opts):
        self._h = C.c_void_p()
        _check(lib().arslam_lm_create(C.byref(self._h), C.byref(make_options(**opts))))

    def close(self):
        if self._h:
            lib().arslam_lm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, **opts):
        _check(lib().arslam_lm_set_options(self._h, C.byref(make_options(**opts))))

    def get_options(self) -> Options:
        o = Options()
        _check(lib().arslam_lm_get_options(self._h, C.byref(o)))
        return o

    def set_iteration_callback(self, fn):
        """ceres::IterationCallback: fn(iteration dict) -> SOLVER_CONTINUE / SOLVER_ABORT /
        SOLVER_TERMINATE_SUCCESSFULLY (None = continue); fn=None removes it."""
        if fn is None:
            self._iter_cb = None
            _check(lib().arslam_lm_set_iteration_callback(self._h, C.cast(None, ITER_CB), None))
            return

        def tramp(ctx, it):
            try:
                d = {f: getattr(it.contents, f) for f, _ in Iteration._fields_}
                r = fn(d)
                return SOLVER_CONTINUE if r is None else int(r)
            except Exception:   # noqa: BLE001 -- a raising callback aborts the solve
                return SOLVER_ABORT
        self._iter_cb = ITER_CB(tramp)
        _check(lib().arslam_lm_set_iteration_callback(self._h, self._iter_cb, None))

    def debug_force_indefinite(self, step_mask):
        """Test hook: linear solves whose bit min(i,63) is set in step_mask see an indefinite
        reduced system (camera diagonal -1), i.e. an invalid LM step."""
        _check(lib().arslam_lm_debug_force_indefinite(self._h, C.c_ulonglong(step_mask & (2**64 - 1))))

    def debug_force_multirank(self, on=True):
        """Test hook: the multi-rank path (split, two-phase factorization, every collective) with
        one rank, so set_comm(0, 1, uid) makes a one-rank RCCL communicator on a one-GPU box."""
        _check(lib().arslam_lm_debug_force_multirank(self._h, 1 if on else 0))

    def set_comm(self, rank, nranks, uid):
        """Join the ranks' exchange: ``uid`` is an RCCL unique id (bytes, one GPU per
        rank) or a host all-reduce ``fn(array, op)`` reducing a numpy array in place
        (op "sum" or "max"), e.g. over torch.distributed gloo."""
        if callable(uid):
            fn = uid

            def tramp(ctx, buf, count, dtype, op):
                try:
                    ct = C.c_double if dtype == 0 else C.c_ubyte
                    arr = np.ctypeslib.as_array(C.cast(buf, C.POINTER(ct)), shape=(count,))
                    fn(arr, "sum" if op == 0 else "max")
                    return 0
                except Exception:   # noqa: BLE001 -- reported to the solver as a comm failure
                    return 1
            self._comm_cb = ALLREDUCE_FN(tramp)
            _check(lib().arslam_lm_set_comm_callback(self._h, rank, nranks, self._comm_cb, None))
        else:
            _check(lib().arslam_lm_set_comm(self._h, rank, nranks, uid))


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().arslam_comm_unique_id(buf))
    return buf.raw


class ResidentProblem(_Handle):
    """SoA problem uploaded once to HBM; ``solve()`` restarts from the loaded state."""

    def __init__(self, camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False,
                 cap_const=None, tag_const=None, comm=None, force_multirank=False, **opts):
        super().__init__(**opts)
        if force_multirank:
            self.debug_force_multirank(True)
        if comm is not None:
            self.set_comm(*comm)
        self.A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
        _check(lib().arslam_lm_load_soa(self._h, C.byref(self.A.s)))

    def solve(self):
        s = Summary()
        _check(lib().arslam_lm_solve_loaded(self._h, C.byref(s)))
        return s.to_dict()

    def owned_captures(self):
        """Indices of the captures this rank owns (every capture on one rank)."""
        n = C.c_int(0)
        _check(lib().arslam_lm_owned_captures(self._h, None, C.c_int(0), C.byref(n)))
        out = (C.c_int * max(n.value, 1))()
        _check(lib().arslam_lm_owned_captures(self._h, out, C.c_int(n.value), C.byref(n)))
        return np.array(out[:n.value], np.int64)

    def debug_break_dependency(self, ticket):
        """Test hook: make one dependency wait of the factorization task graph unreachable."""
        out = C.c_long(-1)
        _check(lib().arslam_lm_debug_break_dependency(self._h, ticket, C.byref(out)))
        return out.value

    @property
    def camera(self):
        return self.A.camera

    @property
    def cap(self):
        return self.A.cap

    @property
    def tag(self):
        return self.A.tag


class Problem(_Handle):
    """ceres::Problem mirror with pointer-keyed parameter blocks (numpy arrays)."""

    def __init__(self, **opts):
        super().__init__(**opts)
        self._keep = []

    @staticmethod
    def _block(a, n):
        if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous
                and a.size == n):
            raise TypeError(f"parameter block must be a C-contiguous float64 array of size {n}")
        return a.ctypes.data_as(_dp)

    def add_residual_block(self, corners, camera, capture, tag):
        c = _f64(corners).reshape(8)
        self._keep += [camera, capture, tag]
        _check(lib().arslam_lm_add_residual_block(self._h, c.ctypes.data_as(_dp),
                                                  self._block(camera, 3), self._block(capture, 6),
                                                  self._block(tag, 6)))

    def set_parameter_block_constant(self, block):
        _check(lib().arslam_lm_set_parameter_block_constant(self._h, block.ctypes.data_as(_dp)))

    def set_parameter_block_variable(self, block):
        _check(lib().arslam_lm_set_parameter_block_variable(self._h, block.ctypes.data_as(_dp)))

    def num_residual_blocks(self):
        return lib().arslam_lm_num_residual_blocks(self._h)

    def solve(self):
        s = Summary()
        _check(lib().arslam_lm_solve(self._h, C.byref(s)))
        return s.to_dict()

    def reset(self):
        _check(lib().arslam_lm_reset(self._h))
        self._keep = []

    def debug_tag_pair_tile(self, tag_a, tag_b):
        """Where the loaded problem's reduced system couples tag blocks a and b: 2 an assembled
        tile, 1 a fill tile of the factor, 0 no tile, -1 not free tags (arslam_lm_debug.h)."""
        st = C.c_int(0)
        _check(lib().arslam_lm_debug_tag_pair_tile(self._h, self._block(tag_a, 6), self._block(tag_b, 6),
                                                   C.byref(st)))
        return st.value


# ---- component entry points (include/arslam_lm_debug.h) ----

def debug_residual_jacobian(cam, cap, tag, corners):
    """Device residuals (n,8) and Jacobians (n,8,15) of n independent observations."""
    cap = _f64(cap, (-1, 6))
    n = cap.shape[0]
    cam = _f64(np.broadcast_to(np.asarray(cam, np.float64), (n, 3)))
    tag = _f64(tag, (-1, 6))
    corners = _f64(corners, (-1, 8))
    r = np.zeros((n, 8))
    J = np.zeros((n, 8, 15))
    _check(lib().arslam_debug_residual_jacobian(n, cam.ctypes.data_as(_dp), cap.ctypes.data_as(_dp),
                                                tag.ctypes.data_as(_dp), corners.ctypes.data_as(_dp),
                                                r.ctypes.data_as(_dp), J.ctypes.data_as(_dp)))
    return r, J


def debug_angle_axis_rotate(w, p):
    """Device AngleAxisRotatePoint of n points: (out (n,3), branch (n,) 1 = Rodrigues, 0 = small angle)."""
    w = _f64(w, (-1, 3))
    p = _f64(p, (-1, 3))
    n = w.shape[0]
    out = np.zeros((n, 3))
    br = np.zeros(n, np.int32)
    _check(lib().arslam_debug_angle_axis_rotate(n, w.ctypes.data_as(_dp), p.ctypes.data_as(_dp),
                                                out.ctypes.data_as(_dp), br.ctypes.data_as(_ip)))
    return out, br


def debug_dense_llt(A, b, executor=0):
    """Device Cholesky + solve of the SPD matrix A (lower triangle used). Returns (L, y, info)."""
    A = _f64(A).copy()
    n = A.shape[0]
    b = _f64(b).reshape(n)
    y = np.zeros(n)
    info = C.c_int(0)
    _check(lib().arslam_debug_dense_llt_ex(C.c_long(n), A.ctypes.data_as(_dp), b.ctypes.data_as(_dp),
                                           y.ctypes.data_as(_dp), C.byref(info), C.c_int(executor)))
    return A, y, info.value


class PlanInfo(C.Structure):
    _fields_ = [("n_reduced", C.c_long), ("n_padded", C.c_long), ("pad_rows", C.c_long),
                ("tiles_per_side", C.c_int), ("n_parts", C.c_int), ("camera_row", C.c_int),
                ("n_levels", C.c_int), ("n_assembled_tiles", C.c_long), ("n_factor_tiles", C.c_long),
                ("n_update_tiles", C.c_long), ("n_update_items", C.c_long), ("n_split_targets", C.c_long),
                ("update_flops", C.c_double), ("n_dag_tasks", C.c_long), ("dag_valid", C.c_int),
                ("factor_flops", C.c_double), ("scalar_flops", C.c_double), ("fill_first_ok", C.c_int)]


def debug_reduced_plan(camera, cap, tag, obs_cap, obs_tag, corners, camera_const=False, cap_const=None,
                       tag_const=None, ordering=2, skip_zero_tiles=1):
    """Host-only symbolic analysis (no device): reduced layout + tile plan.  Returns (info dict, tag_row)."""
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
    info = PlanInfo()
    tag_row = np.zeros(max(A.tag.shape[0], 1), np.int32)
    _check(lib().arslam_debug_reduced_plan(C.byref(A.s), ordering, skip_zero_tiles, C.byref(info),
                                           tag_row.ctypes.data_as(_ip)))
    return {f: getattr(info, f) for f, _ in PlanInfo._fields_}, tag_row[:A.tag.shape[0]]


def debug_reduced_plan_side(camera, cap, tag, obs_cap, obs_tag, corners=None, elimination=ELIM_CAPTURES):
    """Host-only: the reduced layout and tile plan of a fresh one-rank load under elimination
    (ELIM_CAPTURES, ELIM_TAGS or ELIM_MIXED).  Returns (side used, info dict)."""
    if corners is None:
        corners = np.zeros((len(obs_cap), 8))
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, False, None, None)
    info = PlanInfo()
    side = lib().arslam_debug_reduced_plan_side(C.byref(A.s), elimination, C.byref(info))
    _check(min(side, 0))
    return side, {f: getattr(info, f) for f, _ in PlanInfo._fields_}


def box_fingerprint(device=0):
    """The device's hand-off round trips (arslam_debug_box_fingerprint), a few ms of GPU time:
    the kind of MI355X box a measurement ran on."""
    out = (C.c_double * 6)()
    _check(lib().arslam_debug_box_fingerprint(int(device), out))
    return {"cas_poll_ns": out[0], "sc1_load_ns": out[1], "wt_store_ack_ns": out[2],
            "pingpong_ns": out[3], "pingpong_xcc": [int(out[4]), int(out[5])]}


def debug_dag_simulate(g, n_workers, seed=1, policy=0, started=None):
    """Host-only: one simulated interleaving of the persistent executor's protocol on g's one-rank
    plan (policy 0 random, 1-3 adversarial; + 16 without the in-flight cap on claimed targets;
    + 32 with round 5's cap, half the grid).  started=k: only k of the n_workers workgroups ever
    start.  True if every task finished, False on a deadlock."""
    A = _Soa(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
    ok = C.c_int(-1)
    if started is None:
        _check(lib().arslam_debug_dag_simulate(C.byref(A.s), int(n_workers), C.c_uint(seed), int(policy),
                                               C.byref(ok)))
    else:
        _check(lib().arslam_debug_dag_simulate_started(C.byref(A.s), int(n_workers), int(started), C.c_uint(seed),
                                                       int(policy), C.byref(ok)))
    return bool(ok.value)


def debug_dag_workgroup_limit(k):
    """Process-wide test knob: later k_factor_dag launches let only their first k workgroups start
    (as if only k were resident); k <= 0 restores the whole grid."""
    _check(lib().arslam_debug_dag_workgroup_limit(int(k)))


def debug_dag_fault_detail(g, rec):
    """Host-only: the text an executor fault carries for fault record rec[8] (lm_internal.h
    DagFaultField) on g's one-rank plan."""
    A = _Soa(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
    r = (C.c_int * 9)(*([int(v) for v in rec] + [0] * (9 - len(rec))))
    buf = C.create_string_buffer(4096)
    _check(lib().arslam_debug_dag_fault_detail(C.byref(A.s), r, buf, len(buf)))
    return buf.value.decode()


def debug_gather_extend(camera, cap, tag, obs_cap, obs_tag, corners, c0):
    """Host-only: the appended-problem Schur gather plan (the first c0 captures' plan extended by the
    rest) against a fresh plan of the whole problem.  Returns (identical, n_destinations)."""
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners)
    same, nd = C.c_int(0), C.c_int(0)
    _check(lib().arslam_debug_gather_extend(C.byref(A.s), c0, C.byref(same), C.byref(nd)))
    return bool(same.value), nd.value


class SplitInfo(C.Structure):
    _fields_ = [("tiles_per_side", C.c_int), ("n_top_cols", C.c_int), ("n_own_cols", C.c_int),
                ("n_top_tiles", C.c_long), ("n_tiles", C.c_long), ("n_dag_tasks", C.c_long),
                ("phase_split", C.c_long), ("dag_valid", C.c_int), ("n_owned_captures", C.c_int),
                ("top_work", C.c_double), ("max_rank_work", C.c_double), ("total_work", C.c_double),
                ("n_active", C.c_int)]


def debug_rank_split(camera, cap, tag, obs_cap, obs_tag, corners, nranks, rank):
    """Host-only: the multi-rank split the solver makes for `rank` of `nranks` (two-phase tile
    plan of that rank, its validity) and every capture's owner.  Returns (info dict, cap_owner)."""
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners)
    info = SplitInfo()
    owner = np.zeros(max(A.cap.shape[0], 1), np.int32)
    _check(lib().arslam_debug_rank_split(C.byref(A.s), nranks, rank, C.byref(info), owner.ctypes.data_as(_ip)))
    return {f: getattr(info, f) for f, _ in SplitInfo._fields_}, owner[:A.cap.shape[0]]


def debug_ceres_e_blocks(camera, cap, tag, obs_cap, obs_tag, corners=None, camera_const=False, cap_const=None,
                         tag_const=None):
    """Host-only: Ceres 2.0's DENSE_SCHUR e-block set (the rule ELIM_AUTO follows), as
    {captures, tags, camera, max_tag_obs}."""
    if corners is None:
        corners = np.zeros((len(obs_cap), 8))
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
    out = np.zeros(4, np.int32)
    _check(lib().arslam_debug_ceres_e_blocks(C.byref(A.s), out.ctypes.data_as(_ip)))
    return dict(captures=int(out[0]), tags=int(out[1]), camera=int(out[2]), max_tag_obs=int(out[3]))


def debug_mixed_groups(camera, cap, tag, obs_cap, obs_tag, corners=None, camera_const=False, cap_const=None,
                       tag_const=None):
    """Host-only: Ceres' e-block set (e_cap, e_tag: 0/1 per capture / tag) and the ELIM_MIXED
    device problem's {groups, f_blocks, direct, max_blk}."""
    if corners is None:
        corners = np.zeros((len(obs_cap), 8))
    A = _Soa(camera, cap, tag, obs_cap, obs_tag, corners, camera_const, cap_const, tag_const)
    out = np.zeros(4, np.int32)
    e_cap = np.zeros(max(A.cap.shape[0], 1), np.uint8)
    e_tag = np.zeros(max(A.tag.shape[0], 1), np.uint8)
    _check(lib().arslam_debug_mixed_groups(C.byref(A.s), out.ctypes.data_as(_ip),
                                           e_cap.ctypes.data_as(C.POINTER(C.c_ubyte)),
                                           e_tag.ctypes.data_as(C.POINTER(C.c_ubyte))))
    return dict(groups=int(out[0]), f_blocks=int(out[1]), direct=int(out[2]), max_blk=int(out[3]),
                e_cap=e_cap[:A.cap.shape[0]], e_tag=e_tag[:A.tag.shape[0]])


# ---- batched localize (include/arslam_localize.h) ----
LOC_SKIPPED = -1


class LocalizeBatchC(C.Structure):
    _fields_ = [("n_query", C.c_int), ("n_tag", C.c_int), ("n_obs", C.c_int),
                ("camera", _dp), ("tag", _dp), ("tag_in_map", _up), ("query_start", _ip),
                ("obs_tag", _ip), ("corners", _dp), ("pose", _dp), ("init_from_map", C.c_int)]


class LocalizeResult(C.Structure):
    _fields_ = [("status", C.c_int), ("rule", C.c_int), ("num_iterations", C.c_int),
                ("num_successful_steps", C.c_int), ("num_unsuccessful_steps", C.c_int),
                ("init_obs", C.c_int), ("initial_cost", C.c_double), ("final_cost", C.c_double)]


def _loc_results(res):
    n = len(res)
    f = {k: np.array([getattr(r, k) for r in res]) for k, _ in LocalizeResult._fields_}
    f["rule_name"] = [RULES.get(r, str(r)) for r in f["rule"]] if n else []
    return f


class _LocArrays:
    def __init__(self, batch, init_from_map, pose):
        self.camera = _f64(batch.camera).copy()
        self.tag = _f64(batch.tag, (-1, 6)).copy()
        self.q_start = np.ascontiguousarray(batch.q_start, np.int32)
        self.obs_tag = np.ascontiguousarray(batch.obs_tag, np.int32)
        self.corners = _f64(batch.corners, (-1, 8))
        nq = self.q_start.shape[0] - 1
        self.pose = np.zeros((nq, 6)) if pose is None else _f64(pose, (-1, 6)).copy()
        tim = getattr(batch, "tag_in_map", None)
        self.tim = None if tim is None else np.ascontiguousarray(tim, np.uint8)
        self.s = LocalizeBatchC(nq, self.tag.shape[0], self.obs_tag.shape[0],
                                self.camera.ctypes.data_as(_dp), self.tag.ctypes.data_as(_dp),
                                None if self.tim is None else self.tim.ctypes.data_as(_up),
                                self.q_start.ctypes.data_as(_ip), self.obs_tag.ctypes.data_as(_ip),
                                self.corners.ctypes.data_as(_dp), self.pose.ctypes.data_as(_dp),
                                int(bool(init_from_map)))


def localize_many(batch, init_from_map=True, pose=None, **opts):
    """localizeMany on the device (one-shot).  ``batch`` has camera, tag, q_start, obs_tag,
    corners, tag_in_map (synth.LocalizeBatch).  Returns (pose (Nq,6), results dict of arrays)."""
    A = _LocArrays(batch, init_from_map, pose)
    res = (LocalizeResult * max(A.s.n_query, 1))()
    _check(lib().arslam_localize_many(C.byref(A.s), C.byref(make_options(**opts)), res))
    return A.pose, _loc_results(res[:A.s.n_query])


class Localizer:
    """Resident batched localizer: load a batch once, solve it many times."""

    def __init__(self, batch, init_from_map=True, pose=None, **opts):
        self._h = C.c_void_p()
        _check(lib().arslam_localizer_create(C.byref(self._h), C.byref(make_options(**opts))))
        self.A = _LocArrays(batch, init_from_map, pose)
        _check(lib().arslam_localizer_load(self._h, C.byref(self.A.s)))
        self.n_query = self.A.s.n_query

    def solve(self, download=True):
        """Returns (pose or None, results or None, kernel_ms)."""
        ms = C.c_double(0.0)
        pose = np.zeros((self.n_query, 6)) if download else None
        res = (LocalizeResult * max(self.n_query, 1))() if download else None
        _check(lib().arslam_localizer_solve(self._h, None if pose is None else pose.ctypes.data_as(_dp),
                                            res, C.byref(ms)))
        return pose, (None if res is None else _loc_results(res[:self.n_query])), ms.value

    def close(self):
        if self._h:
            lib().arslam_localizer_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- ArSlamSolver host mirror (include/arslam_slam.h) ----
class Transform(C.Structure):
    _fields_ = [("child_frame_id", C.c_char * 128), ("translation", C.c_double * 3),
                ("rotation", C.c_double * 4)]


class SlamSolver:
    """ArSlamSolver (ar_slam_util.hpp:361-497) over the C++ host mirror: captures, arucos and
    blocks addressed by index; uids / ids are strings."""

    def __init__(self, verbose=False, **opts):
        self._h = C.c_void_p()
        _check(lib().arslam_slam_create(C.byref(self._h), C.byref(make_options(**opts))))
        lib().arslam_slam_set_verbose(self._h, int(bool(verbose)))

    def close(self):
        if self._h:
            lib().arslam_slam_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_yaml(self, path):
        _check(lib().arslam_slam_load_yaml(self._h, str(path).encode()))

    def load_yaml_string(self, text):
        _check(lib().arslam_slam_load_yaml_string(self._h, text.encode()))

    def save_yaml(self, path):
        _check(lib().arslam_slam_save_yaml(self._h, str(path).encode()))

    def add_detections(self, capture_uid, ids, corners, image_width=1020, image_height=768, image_path=""):
        """Detections.msg -> capture index, or None when ignored (addDetections :591-627)."""
        corners = _f64(corners, (-1, 8))
        n = corners.shape[0]
        if len(ids) != n:
            raise ValueError("one id per detection")
        arr = (C.c_char_p * max(n, 1))(*[str(i).encode() for i in ids])
        idx = C.c_int(-1)
        _check(lib().arslam_slam_add_detections(self._h, str(capture_uid).encode(), C.c_int(image_width),
                                                C.c_int(image_height), str(image_path).encode(), C.c_int(n),
                                                arr, corners.ctypes.data_as(_dp), C.byref(idx)))
        return None if idx.value < 0 else idx.value

    def solve(self):
        _check(lib().arslam_slam_solve(self._h))

    def solve_incremental(self):
        _check(lib().arslam_slam_solve_incremental(self._h))

    def localize_many(self, first_loc_cap_idx):
        _check(lib().arslam_slam_localize_many(self._h, C.c_int(first_loc_cap_idx)))

    @property
    def num_captures(self):
        return lib().arslam_slam_num_captures(self._h)

    @property
    def num_arucos(self):
        return lib().arslam_slam_num_arucos(self._h)

    @property
    def num_blocks(self):
        return lib().arslam_slam_num_blocks(self._h)

    @property
    def num_solves(self):
        return lib().arslam_slam_num_solves(self._h)

    def last_summary(self):
        s = Summary()
        _check(lib().arslam_slam_last_summary(self._h, C.byref(s)))
        return s.to_dict()

    def solve_summary(self, i):
        """Summary of optimize() call i."""
        s = Summary()
        _check(lib().arslam_slam_solve_summary(self._h, C.c_int(i), C.byref(s)))
        return s.to_dict()

    def solve_capture(self, i):
        """Index of the capture whose optimize() was call i (the drivers' visiting order)."""
        c = C.c_int(-1)
        _check(lib().arslam_slam_solve_capture(self._h, C.c_int(i), C.byref(c)))
        return c.value

    def solve_order(self):
        return [self.solve_capture(i) for i in range(self.num_solves)]

    def unsolved_captures(self):
        """The unsolved-capture set in its iteration order (begin() first)."""
        n = C.c_int(0)
        _check(lib().arslam_slam_unsolved_captures(self._h, None, C.c_int(0), C.byref(n)))
        out = (C.c_int * max(n.value, 1))()
        _check(lib().arslam_slam_unsolved_captures(self._h, out, C.c_int(n.value), C.byref(n)))
        return [int(out[i]) for i in range(n.value)]

    def capture(self, c):
        buf = C.create_string_buffer(256)
        pose = np.zeros(6)
        _check(lib().arslam_slam_capture(self._h, C.c_int(c), buf, C.c_int(256), pose.ctypes.data_as(_dp)))
        return buf.value.decode(), pose

    def set_capture_pose(self, c, pose):
        p = _f64(pose).reshape(6).copy()
        _check(lib().arslam_slam_set_capture_pose(self._h, C.c_int(c), p.ctypes.data_as(_dp)))

    def aruco(self, a):
        buf = C.create_string_buffer(256)
        pose = np.zeros(6)
        init = C.c_int(0)
        _check(lib().arslam_slam_aruco(self._h, C.c_int(a), buf, C.c_int(256), pose.ctypes.data_as(_dp),
                                       C.byref(init)))
        return buf.value.decode(), pose, bool(init.value)

    def set_aruco_pose(self, a, pose):
        p = _f64(pose).reshape(6).copy()
        _check(lib().arslam_slam_set_aruco_pose(self._h, C.c_int(a), p.ctypes.data_as(_dp)))

    def block(self, b):
        c, a, added = C.c_int(), C.c_int(), C.c_int()
        rect = np.zeros(8)
        _check(lib().arslam_slam_block(self._h, C.c_int(b), C.byref(c), C.byref(a), rect.ctypes.data_as(_dp),
                                       C.byref(added)))
        return c.value, a.value, rect, bool(added.value)

    def camera(self):
        p = np.zeros(3)
        w, h = C.c_int(), C.c_int()
        _check(lib().arslam_slam_camera(self._h, p.ctypes.data_as(_dp), C.byref(w), C.byref(h)))
        return p, (None if w.value < 0 else (w.value, h.value))

    def set_camera(self, params):
        p = _f64(params).reshape(3).copy()
        _check(lib().arslam_slam_set_camera(self._h, p.ctypes.data_as(_dp)))

    def capture_poses(self):
        return np.array([self.capture(c)[1] for c in range(self.num_captures)]).reshape(-1, 6)

    def aruco_poses(self):
        return np.array([self.aruco(a)[1] for a in range(self.num_arucos)]).reshape(-1, 6)

    def get_transforms(self):
        n = C.c_int(0)
        _check(lib().arslam_slam_get_transforms(self._h, None, C.c_int(0), C.byref(n)))
        arr = (Transform * max(n.value, 1))()
        _check(lib().arslam_slam_get_transforms(self._h, arr, C.c_int(n.value), C.byref(n)))
        return [(t.child_frame_id.decode(), np.array(t.translation[:]), np.array(t.rotation[:]))
                for t in arr[:n.value]]

    def camera_info(self):
        k, p = np.zeros(9), np.zeros(12)
        _check(lib().arslam_slam_camera_info(self._h, k.ctypes.data_as(_dp), p.ctypes.data_as(_dp)))
        return k.reshape(3, 3), p.reshape(3, 4)
