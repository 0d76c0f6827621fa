"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
symbol the headers declare, and its host-side logic behaves without a GPU
(argument validation, Ceres-style problem building, loud failure instead of
a CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from ar_slam_amd import build, lm
    build.build()
    return lm


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(arslam_\w+)\s*\(", src)))


@pytest.mark.parametrize("header", ["arslam_lm.h", "arslam_lm_debug.h"])
def test_library_exports_every_declared_symbol(L, header):
    lib = C.CDLL(L.library_path())
    names = _declared(header)
    assert names
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/{header} but not exported"
    for n in names:
        assert n in L.EXPORTS


def test_options_defaults_are_the_reference_settings(L):
    o = L.make_options()
    assert o.max_num_iterations == 50               # ar_slam_util.cpp:1004
    assert o.function_tolerance == 1e-6 and o.gradient_tolerance == 1e-10
    assert o.parameter_tolerance == 1e-8 and o.initial_trust_region_radius == 1e4
    assert o.min_lm_diagonal == 1e-6 and o.max_lm_diagonal == 1e32
    assert o.max_num_consecutive_invalid_steps == 5 and o.jacobi_scaling == 1
    with pytest.raises(AttributeError):
        L.make_options(no_such_option=1)


def test_summary_struct_matches_header(L):
    # ctypes mirror of arslam_lm_summary must be the size the library expects:
    # a mismatch would corrupt memory, so check the field order against the header
    src = open(os.path.join(ROOT, "include", "arslam_lm.h")).read()
    body = src[src.index("typedef struct {\n  int termination;"):src.index("} arslam_lm_summary;")]
    fields = re.findall(r"\b(\w+)(?:\[[^\]]*\])?\s*[;,]", re.sub(r"/\*.*?\*/", "", body, flags=re.S))
    fields = [f for f in fields if f not in ("int", "double", "long")]
    ours = [f for f, _ in L.Summary._fields_]
    assert ours == fields


def test_problem_building_and_validation(L):
    prob = L.Problem()
    cam = np.array([900.0, 0.0, 0.0])
    caps = [np.zeros(6) for _ in range(2)]
    tags = [np.zeros(6) for _ in range(3)]
    prob.add_residual_block(np.zeros(8), cam, caps[0], tags[0])
    prob.add_residual_block(np.zeros(8), cam, caps[1], tags[2])
    assert prob.num_residual_blocks() == 2
    with pytest.raises(L.LMError):           # second camera block: unsupported
        prob.add_residual_block(np.zeros(8), np.zeros(3), caps[0], tags[0])
    with pytest.raises(L.LMError):           # capture reused as a tag
        prob.add_residual_block(np.zeros(8), cam, caps[0], caps[1])
    with pytest.raises(L.LMError):           # not part of the problem
        prob.set_parameter_block_constant(np.zeros(6))
    prob.set_parameter_block_constant(tags[0])
    prob.reset()
    assert prob.num_residual_blocks() == 0
    with pytest.raises(TypeError):
        prob.add_residual_block(np.zeros(8), cam, np.zeros(5), tags[0])


def test_solve_without_gpu_fails_loudly(L):
    if L.device_count() > 0:
        pytest.skip("a GPU is present")
    from ar_slam_amd import synth
    g = synth.config_graph("tiny")
    with pytest.raises(L.LMError):
        L.solve_graph(g)


def test_empty_problem_converges_immediately(L):
    s = L.Problem().solve()
    assert s["termination"] == "CONVERGENCE" and s["num_linear_solves"] == 0


def test_set_and_get_options_roundtrip(L):
    """Per-solve options (ArSlamSolver::optimize builds Solver::Options per call, ar_slam_util.cpp:1003-1012)."""
    prob = L.Problem()
    prob.set_options(max_num_iterations=7, minimizer_progress_to_stdout=1, function_tolerance=1e-9)
    o = prob.get_options()
    assert o.max_num_iterations == 7 and o.minimizer_progress_to_stdout == 1
    assert o.function_tolerance == 1e-9
    with pytest.raises(L.LMError):
        prob.set_options(max_num_iterations=-1)
    with pytest.raises(L.LMError):
        prob.set_options(elimination=5)
    assert prob.get_options().max_num_iterations == 7   # a rejected call leaves the options unchanged
