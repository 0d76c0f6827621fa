"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Tolerances (fp64 everywhere; the oracle restates Ceres' arithmetic, the
device sums in a different order and scatters the reduced system with
atomics, so agreement is to rounding, not bitwise):
  * residual / Jacobian rows: 1e-12 relative to the row scale;
  * dense Cholesky solve: 1e-10 relative residual on SPD test matrices;
  * LM traces: per-iteration cost 1e-9 relative for the first 5 iterations,
    final cost 1e-8 relative, same termination type and rule, iteration
    count +-1, focal 1e-8 relative; every capture and tag pose after one rigid
    gauge alignment fitted on the tags: positions 1e-6 m, rotations 1e-7 rad
    (tests/gauge.py; SURVEY.md §8c proposal).
"""
import numpy as np
import pytest

from ar_slam_amd import synth
from gauge import assert_poses_match, load_cfg3_golden

pytestmark = pytest.mark.gpu


def _random_obs(rng, n):
    cam = np.stack([rng.uniform(500, 3000, n), np.zeros(n), np.zeros(n)], 1)
    tag = np.concatenate([rng.normal(0, 1, (n, 3)), rng.normal(0, 1, (n, 3))], 1)
    w = rng.normal(0, 1, (n, 3)) * rng.choice([1.0, 1e-2, 0.0, 3.0], (n, 1))
    cap = np.concatenate([-tag[:, :3] + rng.normal(0, 0.2, (n, 3)) + [0, 0, 1.0], w], 1)
    tag[::5, 3:] = 0.0          # small-angle branch exactly at w = 0
    corners = rng.normal(0, 100, (n, 8))
    return cam, cap, tag, corners


def test_residual_jacobian_matches_oracle(lm, oracle):
    rng = np.random.default_rng(7)
    cam, cap, tag, corners = _random_obs(rng, 512)
    r, J = lm.debug_residual_jacobian(cam, cap, tag, corners)
    for i in range(cam.shape[0]):
        ro, Jo = oracle.residual_jacobian(cam[i], cap[i], tag[i], corners[i])
        np.testing.assert_allclose(r[i], ro, rtol=1e-12, atol=1e-9)
        scale = np.abs(Jo).max(axis=1, keepdims=True) + 1e-300
        assert np.max(np.abs(J[i] - Jo) / scale) < 1e-12
    # the capture- and tag-translation columns are the same numbers (the stored Jacobian keeps them once)
    assert np.array_equal(J[..., 3:6], J[..., 9:12])   # ([f, 0, 0, t_c, w_c, t_t, w_t])


@pytest.mark.parametrize("executor", [0, 1])
@pytest.mark.parametrize("n", [5, 64, 200, 777])
def test_dense_llt_matches_numpy(lm, n, executor):
    """Tiled Cholesky + forward/backward solve of a dense SPD matrix: level launches (0) and the
    persistent factorization + persistent backward solve (1)."""
    rng = np.random.default_rng(n)
    B = rng.normal(size=(n, n))
    A = B @ B.T + n * np.eye(n)
    b = rng.normal(size=n)
    L, y, info = lm.debug_dense_llt(A, b, executor=executor)
    assert info == 0
    Lref = np.linalg.cholesky(A)
    np.testing.assert_allclose(L, Lref, rtol=1e-10, atol=1e-10 * np.abs(Lref).max())
    np.testing.assert_allclose(A @ y, b, rtol=1e-9, atol=1e-9 * np.abs(b).max())


@pytest.mark.parametrize("executor", [0, 1])
def test_dense_llt_reports_indefinite(lm, executor):
    A = np.eye(100)
    A[70, 70] = -1.0
    _, _, info = lm.debug_dense_llt(A, np.ones(100), executor=executor)
    assert info == 71


def _compare_solves(g, ours, ref, n_cost_iters=5):
    cam_o, cap_o, tag_o, s_o = ours
    cam_r, cap_r, tag_r, s_r = ref
    assert s_o["termination"] == s_r["termination"]
    assert s_o["rule"] == s_r["rule"]
    assert abs(len(s_o["iterations"]) - len(s_r["iterations"])) <= 1
    co = [it["cost"] for it in s_o["iterations"]]
    cr = [it["cost"] for it in s_r["iterations"]]
    for a, b in list(zip(co, cr))[:n_cost_iters]:
        assert abs(a - b) <= 1e-9 * abs(b), (co, cr)
    assert abs(s_o["final_cost"] - s_r["final_cost"]) <= 1e-8 * s_r["final_cost"]
    assert abs(cam_o[0] - cam_r[0]) <= 1e-8 * cam_r[0]
    # every capture and tag pose (positions and rotations), in the oracle's gauge
    assert_poses_match(cap_o, tag_o, cap_r, tag_r, tags=np.unique(g.obs_tag), caps=np.unique(g.obs_cap))


@pytest.mark.parametrize("name", ["tiny", "small", "medium", "cfg2", "wide"])
def test_lm_solve_matches_oracle(lm, oracle, name):
    """(wide: camera roll and tag yaw ~ U(-pi, pi), SURVEY.md §8d -- angle-axis up to |w| ~ pi)"""
    g = synth.config_graph(name)
    ref = oracle.solve_graph(g)
    ours = lm.solve_graph(g)
    _compare_solves(g, ours, ref)
    assert ours[3]["termination"] == "CONVERGENCE"


def test_pointer_api_matches_soa(lm):
    """Problem (AddResidualBlock / Solve, caller-owned blocks) == bulk SoA path."""
    g = synth.config_graph("small")
    camera = g.camera.copy()
    caps = [g.cap[c].copy() for c in range(g.n_cap)]
    tags = [g.tag[t].copy() for t in range(g.n_tag)]
    prob = lm.Problem()
    for b in range(g.n_obs):
        prob.add_residual_block(g.corners[b], camera, caps[g.obs_cap[b]], tags[g.obs_tag[b]])
    assert prob.num_residual_blocks() == g.n_obs
    s = prob.solve()
    cam2, cap2, tag2, s2 = lm.solve_graph(g)
    assert s["termination"] == s2["termination"]
    assert abs(s["final_cost"] - s2["final_cost"]) <= 1e-10 * s2["final_cost"]
    np.testing.assert_allclose(camera, cam2, rtol=1e-10)
    np.testing.assert_allclose(np.stack(caps), cap2, rtol=1e-8, atol=1e-9)


def test_pointer_api_resolve_reuses_the_resident_problem(lm):
    """Solving an unchanged pointer-keyed problem again reloads only the parameter values (no
    host rebuild, no plan, no observation upload: setup_kind VALUES), from the caller's current
    block values, and gives exactly what a fresh problem gives from those values."""
    g = synth.config_graph("small")
    camera = g.camera.copy()
    caps = [g.cap[c].copy() for c in range(g.n_cap)]
    tags = [g.tag[t].copy() for t in range(g.n_tag)]
    prob = lm.Problem()
    for b in range(g.n_obs):
        prob.add_residual_block(g.corners[b], camera, caps[g.obs_cap[b]], tags[g.obs_tag[b]])
    s1 = prob.solve()
    # perturb the solved state in the caller's blocks, solve again (same structure)
    camera[0] *= 1.02
    for c in caps:
        c[:3] += 0.01
    start = (camera.copy(), np.stack(caps).copy(), np.stack(tags).copy())
    s2 = prob.solve()
    assert s1["setup_kind"] == lm.SETUP_LOAD
    assert s2["setup_kind"] == lm.SETUP_VALUES
    fresh = lm.Problem()
    cam_f = start[0].copy()
    caps_f = [c.copy() for c in start[1]]
    tags_f = [t.copy() for t in start[2]]
    for b in range(g.n_obs):
        fresh.add_residual_block(g.corners[b], cam_f, caps_f[g.obs_cap[b]], tags_f[g.obs_tag[b]])
    s3 = fresh.solve()
    assert [i["cost"] for i in s2["iterations"]] == [i["cost"] for i in s3["iterations"]]
    np.testing.assert_array_equal(camera, cam_f)
    # a structural change (a block held constant) rebuilds
    prob.set_parameter_block_constant(tags[0])
    s4 = prob.solve()
    assert s4["setup_kind"] == lm.SETUP_LOAD


def test_appended_problem_keeps_plan_and_matches_a_fresh_load(lm, oracle):
    """solveIncremental's growth (ar_slam_util.cpp:720-736): residual blocks of new captures that
    see only known tags are appended to the resident problem.  When their tile pairs are in the
    loaded pattern the layout, elimination order and factorization plan are kept
    (setup_kind APPEND: only the capture side, the gather plan and the values are uploaded), and
    the solve gives the trace a fresh load of the grown problem gives, and the oracle's."""
    g = synth.config_graph("cfg2")
    camera = g.camera.copy()
    caps = [g.cap[c].copy() for c in range(g.n_cap)]
    tags = [g.tag[t].copy() for t in range(g.n_tag)]
    prob = lm.Problem(elimination=lm.ELIM_CAPTURES)
    first = 700
    seen = set()
    for b in range(g.n_obs):
        if g.obs_cap[b] < first:
            prob.add_residual_block(g.corners[b], camera, caps[g.obs_cap[b]], tags[g.obs_tag[b]])
            seen.add(int(g.obs_tag[b]))
    s1 = prob.solve()
    assert s1["setup_kind"] == lm.SETUP_LOAD
    # append later captures whose tags are all known and were seen together before (their
    # blocks of the reduced system are then tiles of the loaded factor)
    pairs = set()
    for c in range(first):
        ts = sorted(set(g.obs_tag[g.obs_cap == c].tolist()))
        pairs.update((a, b) for a in ts for b in ts if a < b)
    added = []
    for c in range(first, g.n_cap):
        ts = sorted(set(g.obs_tag[g.obs_cap == c].tolist()))
        if set(ts) <= seen and all((a, b) in pairs for a in ts for b in ts if a < b):
            added.append(c)
    added = added[:20]
    assert len(added) >= 5
    for c in added:
        for b in np.nonzero(g.obs_cap == c)[0]:
            prob.add_residual_block(g.corners[b], camera, caps[c], tags[g.obs_tag[b]])
    start = (camera.copy(), [c.copy() for c in caps], [t.copy() for t in tags])
    s2 = prob.solve()
    assert s2["setup_kind"] == lm.SETUP_APPEND, s2["setup_kind"]   # (the plan was kept: no timing check)
    # a fresh problem of the same blocks, from the same values
    fresh = lm.Problem(elimination=lm.ELIM_CAPTURES)
    cam_f, caps_f, tags_f = start[0].copy(), [c.copy() for c in start[1]], [t.copy() for t in start[2]]
    order = [b for b in range(g.n_obs) if g.obs_cap[b] < first] + \
        [b for c in added for b in np.nonzero(g.obs_cap == c)[0]]
    for b in order:
        fresh.add_residual_block(g.corners[b], cam_f, caps_f[g.obs_cap[b]], tags_f[g.obs_tag[b]])
    s3 = fresh.solve()
    assert s3["setup_kind"] == lm.SETUP_LOAD
    assert [i["step_is_successful"] for i in s2["iterations"]] == [i["step_is_successful"] for i in s3["iterations"]]
    for a, b in zip(s2["iterations"], s3["iterations"]):
        assert abs(a["cost"] - b["cost"]) <= 1e-9 * b["cost"]
    assert abs(camera[0] - cam_f[0]) <= 1e-8 * cam_f[0]
    # and the oracle on the grown problem from the same start
    cap_ids = sorted({int(g.obs_cap[b]) for b in order})
    cpos = {c: i for i, c in enumerate(cap_ids)}
    tag_ids = sorted({int(g.obs_tag[b]) for b in order})
    tpos = {t: i for i, t in enumerate(tag_ids)}
    _, _, _, so = oracle.solve(start[0].copy(), np.array([start[1][c] for c in cap_ids]),
                               np.array([start[2][t] for t in tag_ids]),
                               np.array([cpos[int(g.obs_cap[b])] for b in order], np.int32),
                               np.array([tpos[int(g.obs_tag[b])] for b in order], np.int32),
                               g.corners[order])
    assert so["termination"] == s2["termination"]
    assert abs(so["final_cost"] - s2["final_cost"]) <= 1e-8 * so["final_cost"]


def test_appended_coupling_in_a_fill_tile_matches_a_fresh_load(lm):
    """An appended capture that couples two known tags never seen together, where their block of
    the reduced system lies in a fill tile of the loaded factor (arslam_lm_debug_tag_pair_tile):
    the plan is kept (setup_kind APPEND: the pair's tile is a fill tile of the loaded factor, which
    k_schur clears every step and the extended gather writes into), and the solve gives
    the trace a fresh load of the grown problem gives, to 1e-9.  The appended captures are
    synthetic: a camera above the midpoint of such a pair (the nearest such pairs, up to 3 m apart;
    2-3.3 m up) sees both tags."""
    g = synth.config_graph("cfg2")
    camera = g.camera.copy()
    first = 700
    caps = [g.cap[c].copy() for c in range(first)]
    tags = [g.tag[t].copy() for t in range(g.n_tag)]
    prob = lm.Problem(elimination=lm.ELIM_CAPTURES)
    seen, pairs = set(), set()
    for c in range(first):
        ts = sorted(set(g.obs_tag[g.obs_cap == c].tolist()))
        seen.update(ts)
        pairs.update((a, b) for a in ts for b in ts if a < b)
    obs = [(g.corners[b], int(g.obs_cap[b]), int(g.obs_tag[b])) for b in range(g.n_obs) if g.obs_cap[b] < first]
    for corners, c, t in obs:
        prob.add_residual_block(corners, camera, caps[c], tags[t])
    s1 = prob.solve()
    assert s1["setup_kind"] == lm.SETUP_LOAD
    xy = g.tag_true[:, :2]
    hist, fill = {}, []
    for a in sorted(seen):
        for b in sorted(seen):
            d = np.linalg.norm(xy[a] - xy[b])
            if a >= b or (a, b) in pairs or d > 3.0:
                continue
            st = prob.debug_tag_pair_tile(tags[a], tags[b])
            hist[st] = hist.get(st, 0) + 1
            if st == 1:
                fill.append((d, a, b))
    picked, used = [], set()
    for d, a, b in sorted(fill):
        if a not in used and b not in used and len(picked) < 6:
            picked.append((a, b))
            used.update((a, b))
    assert picked, f"no unseen tag pair in a fill tile (pair statuses {hist})"
    rng = np.random.default_rng(5)
    for a, b in picked:
        mid = 0.5 * (g.tag_true[a, :3] + g.tag_true[b, :3])
        h = max(2.0, 1.1 * np.linalg.norm(xy[a] - xy[b]))
        pose = np.array([-mid[0], -mid[1], h, 0.0, 0.0, 0.0])   # centre (mid, -h), looking along +z
        cor = synth.project_corners(g.camera_true, np.tile(pose, (2, 1)), g.tag_true[[a, b]])
        assert np.abs(cor[:, 0::2]).max() < 0.5 * synth.IMG_W and np.abs(cor[:, 1::2]).max() < 0.5 * synth.IMG_H
        cor = cor + rng.normal(0.0, 0.5, cor.shape)
        caps.append(pose + np.concatenate([rng.normal(0, 0.02, 3), rng.normal(0, 0.02, 3)]))
        for row, t in zip(cor, (a, b)):
            obs.append((np.ascontiguousarray(row), len(caps) - 1, t))
            prob.add_residual_block(obs[-1][0], camera, caps[-1], tags[t])
    start = (camera.copy(), [c.copy() for c in caps], [t.copy() for t in tags])
    s2 = prob.solve()
    assert s2["setup_kind"] == lm.SETUP_APPEND, s2["setup_kind"]
    fresh = lm.Problem(elimination=lm.ELIM_CAPTURES)
    cam_f, caps_f, tags_f = start[0].copy(), [c.copy() for c in start[1]], [t.copy() for t in start[2]]
    for corners, c, t in obs:
        fresh.add_residual_block(corners, cam_f, caps_f[c], tags_f[t])
    s3 = fresh.solve()
    assert s3["setup_kind"] == lm.SETUP_LOAD
    print(f"appended {len(picked)} captures coupling unseen tag pairs in fill tiles (statuses {hist})")
    assert [i["step_is_successful"] for i in s2["iterations"]] == [i["step_is_successful"] for i in s3["iterations"]]
    for x, y in zip(s2["iterations"], s3["iterations"]):
        assert abs(x["cost"] - y["cost"]) <= 1e-9 * y["cost"]
    assert abs(camera[0] - cam_f[0]) <= 1e-8 * cam_f[0]


def test_localize_constant_map(lm, oracle):
    """localizeOne: tags and camera constant (ar_slam_util.cpp:965,972), one free capture each."""
    g = synth.config_graph("medium")
    tag_const = np.ones(g.n_tag, np.uint8)
    kw = dict(camera_const=True, tag_const=tag_const)
    cam_t = g.camera_true.copy()
    ref = oracle.solve(cam_t, g.cap, g.tag_true, g.obs_cap, g.obs_tag, g.corners, **kw)
    ours = lm.solve_soa(cam_t, g.cap, g.tag_true, g.obs_cap, g.obs_tag, g.corners, **kw)
    assert ours[3]["termination"] == ref[3]["termination"]
    assert abs(ours[3]["final_cost"] - ref[3]["final_cost"]) <= 1e-8 * ref[3]["final_cost"]
    np.testing.assert_allclose(ours[1], ref[1], rtol=1e-7, atol=1e-8)
    np.testing.assert_array_equal(ours[2], g.tag_true)   # constant blocks untouched
    assert ours[0][0] == cam_t[0]


def test_edge_cases_match_oracle(lm, oracle):
    """Unobserved tag, duplicate tag in one capture, a constant capture, empty capture."""
    g = synth.config_graph("small")
    obs_cap = np.concatenate([g.obs_cap, [3]]).astype(np.int32)
    obs_tag = np.concatenate([g.obs_tag, [g.obs_tag[8 * 3]]]).astype(np.int32)   # duplicate
    corners = np.concatenate([g.corners, g.corners[8 * 3:8 * 3 + 1] + 0.3])
    tag = np.concatenate([g.tag, [[9.0, 9.0, 0.0, 0.0, 0.0, 0.3]]])            # unobserved
    cap = np.concatenate([g.cap, [[0.0, 0.0, -1.0, 3.1, 0.0, 0.0]]])            # no observations
    cap_const = np.zeros(cap.shape[0], np.uint8)
    cap_const[5] = 1
    kw = dict(cap_const=cap_const)
    ref = oracle.solve(g.camera, cap, tag, obs_cap, obs_tag, corners, **kw)
    ours = lm.solve_soa(g.camera, cap, tag, obs_cap, obs_tag, corners, **kw)
    assert ours[3]["termination"] == ref[3]["termination"]
    assert abs(ours[3]["final_cost"] - ref[3]["final_cost"]) <= 1e-8 * ref[3]["final_cost"]
    np.testing.assert_array_equal(ours[1][5], cap[5])
    np.testing.assert_array_equal(ours[1][-1], cap[-1])
    np.testing.assert_array_equal(ours[2][-1], tag[-1])


def test_resident_problem_resolves_identically(lm):
    g = synth.config_graph("medium")
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
    s1 = rp.solve()
    c1 = rp.cap.copy()
    s2 = rp.solve()
    assert [i["cost"] for i in s1["iterations"]] == pytest.approx([i["cost"] for i in s2["iterations"]], rel=1e-12)
    np.testing.assert_allclose(rp.cap, c1, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("ordering", [0, 1, 2])
@pytest.mark.parametrize("skip", [0, 1])
@pytest.mark.parametrize("name", ["small", "cfg2"])
def test_reduced_orderings_match_oracle(lm, oracle, name, skip, ordering):
    """Natural / RCM / nested-dissection reduced orderings, dense or zero-tile-skipping plans."""
    g = synth.config_graph(name)
    ref = oracle.solve_graph(g)
    ours = lm.solve_graph(g, cholesky_skip_zero_tiles=skip, reduced_ordering=ordering)
    _compare_solves(g, ours, ref)
    if name == "cfg2" and skip:
        s = ours[3]
        T = (s["n_reduced"] + 1 + 63) // 64
        assert s["n_factor_tiles"] < T * (T + 1) // 2
    if ordering == 2 and skip and name == "cfg2":
        # nested dissection: the tile elimination tree is much shallower than the chain
        assert ours[3]["n_levels"] < (ours[3]["n_reduced"] + 64) // 64 // 2


def test_sparse_plan_equals_dense_plan_on_same_order(lm):
    """Skipping zero tiles changes nothing but the work: the trace matches the dense plan."""
    g = synth.config_graph("cfg2")
    dense = lm.solve_graph(g, cholesky_skip_zero_tiles=0, reduced_ordering=1)
    sparse = lm.solve_graph(g, cholesky_skip_zero_tiles=1, reduced_ordering=1)
    cd = [it["cost"] for it in dense[3]["iterations"]]
    cs = [it["cost"] for it in sparse[3]["iterations"]]
    assert len(cd) == len(cs)
    np.testing.assert_allclose(cs, cd, rtol=1e-10)


def test_cfg3_matches_golden_oracle_trace(lm):
    """The headline workload (10k captures / 2k tags) against the oracle's committed trace and
    final state: every capture and tag pose, gauge-aligned on the tags."""
    gold, final = load_cfg3_golden()
    g = synth.config_graph("cfg3")
    cam, cap, tag, s = lm.solve_graph(g)
    assert s["termination"] == gold["termination"] and s["rule"] == gold["rule"]
    assert abs(s["num_linear_solves"] - gold["num_linear_solves"]) <= 1
    costs = [it["cost"] for it in s["iterations"]]
    for a, b in list(zip(costs, gold["cost"]))[:5]:
        assert abs(a - b) <= 1e-9 * abs(b), (costs, gold["cost"])
    np.testing.assert_allclose([it["trust_region_radius"] for it in s["iterations"]][:5],
                               gold["trust_region_radius"][:5], rtol=1e-12)
    assert abs(s["final_cost"] - gold["final_cost"]) <= 1e-8 * gold["final_cost"]
    assert abs(cam[0] - gold["final_focal"]) <= 1e-8 * gold["final_focal"]
    assert abs(s["final_rms_px"] - gold["final_rms_px"]) <= 1e-8 * gold["final_rms_px"]
    assert abs(cam[0] - final["camera"][0]) <= 1e-8 * final["camera"][0]
    e = assert_poses_match(cap, tag, final["cap"], final["tag"])
    print("cfg3 pose errors vs the oracle:", e)


@pytest.mark.parametrize("name", ["medium", "cfg2"])
@pytest.mark.parametrize("ordering", [1, 2])
def test_persistent_executor_matches_level_launches(lm, oracle, name, ordering):
    """The persistent task-graph factorization (default) and the level-synchronous one give the
    same LM trace (both against the oracle's tolerances)."""
    g = synth.config_graph(name)
    ref = oracle.solve_graph(g)
    lev = lm.solve_graph(g, factor_executor=0, reduced_ordering=ordering)
    dag = lm.solve_graph(g, factor_executor=1, reduced_ordering=ordering)
    _compare_solves(g, lev, ref)
    _compare_solves(g, dag, ref)
    cl = [it["cost"] for it in lev[3]["iterations"]]
    cd = [it["cost"] for it in dag[3]["iterations"]]
    assert len(cl) == len(cd)
    np.testing.assert_allclose(cd, cl, rtol=1e-10)


def test_cfg3_repeated_solves_are_bit_identical(lm):
    """The device path is deterministic (no atomics in any sum that reaches the step, fixed
    summation orders in the task-graph factorization): repeated solves of the headline
    workload from the same HBM-resident state give bit-identical traces and parameters.
    A data race in the persistent executor shows up here as a differing bit."""
    g = synth.config_graph("cfg3")
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
    ref = rp.solve()
    tags = rp.tag.copy()
    for _ in range(3):
        s = rp.solve()
        assert [i["cost"] for i in s["iterations"]] == [i["cost"] for i in ref["iterations"]]
        assert [i["trust_region_radius"] for i in s["iterations"]] == \
            [i["trust_region_radius"] for i in ref["iterations"]]
        assert np.array_equal(rp.tag, tags)


def test_executor_grid_size_does_not_change_the_result(lm, monkeypatch):
    """The persistent factorization sums every tile in a fixed order whatever the grid, so any
    number of workgroups gives bit-identical steps.  Small grids also exercise the claim cap
    (claimed continuation targets in flight <= half the grid; with one workgroup, none) and the
    deadlock-freedom of the ticket order with few workers."""
    g = synth.config_graph("cfg2")
    cam, cap, tag, ref = lm.solve_graph(g)
    for grid in ("1", "3", "64"):
        monkeypatch.setenv("ARSLAM_DAG_GRID", grid)
        c2, p2, t2, s = lm.solve_graph(g)
        assert [i["cost"] for i in s["iterations"]] == [i["cost"] for i in ref["iterations"]], grid
        assert np.array_equal(t2, tag) and np.array_equal(p2, cap) and np.array_equal(c2, cam), grid


@pytest.mark.parametrize("name", ["cfg2", "cfg3"])
def test_factorization_completes_with_few_resident_workgroups(lm, name):
    """Progress independent of residency: the launch keeps its full grid (448
    workgroups on cfg3) but only the first k workgroups ever start -- the rest return at once, as
    when another process or other ranks hold the GPU.  The claim cap is half the workgroups that
    have started (k = 1: no claims; 2: one; 7: three), so every factorization finishes, and the
    fixed summation order makes the solve bit-identical to the whole grid's."""
    g = synth.config_graph(name)
    cam, cap, tag, ref = lm.solve_graph(g)
    try:
        for k in (1, 2, 7):
            lm.debug_dag_workgroup_limit(k)
            c2, p2, t2, s = lm.solve_graph(g)
            assert [i["cost"] for i in s["iterations"]] == [i["cost"] for i in ref["iterations"]], k
            assert np.array_equal(t2, tag) and np.array_equal(p2, cap) and np.array_equal(c2, cam), k
    finally:
        lm.debug_dag_workgroup_limit(0)


@pytest.mark.parametrize("side", ["captures", "tags", "auto"])
@pytest.mark.parametrize("name", ["kvar", "k24", "wall"])
def test_large_captures_match_oracle(lm, oracle, name, side):
    """Captures of 8 to 120 tags (the reference adds every block of a capture, ar_slam_util.cpp:704-731,
    and seeds solve() from the capture with the most tags, :759-771): kvar mixes captures of 8, 11,
    16, 40 and 64 tags with one of 80, k24 has 24 per capture, wall 10 captures of 120.  Captures of
    more than 10 tags take k_schur's second launch (its LDS sized for them); every per-capture kernel
    takes the rows in chunks of 8 observations.  Under tag elimination the e-blocks are tags seen by
    up to 20 captures."""
    g = synth.config_graph(name)
    elim = {"auto": lm.ELIM_AUTO, "captures": lm.ELIM_CAPTURES, "tags": lm.ELIM_TAGS}[side]
    ref = oracle.solve_graph(g)
    ours = lm.solve_graph(g, elimination=elim)
    _compare_solves(g, ours, ref)
    assert ours[3]["termination"] == "CONVERGENCE"
    if side == "captures":
        assert ours[3]["elimination_used"] == lm.ELIM_CAPTURES


def test_capture_of_more_than_256_tags(lm, oracle):
    """A capture seeing more distinct tags than one wave's LDS holds (kMaxSchurBlocks = 256; every
    ArUco dictionary the reference supports has at most 250 ids) cannot be an e-block: explicit
    capture elimination reports ARSLAM_E_UNSUPPORTED, and ARSLAM_ELIM_AUTO eliminates the tags
    instead and matches the oracle."""
    g = synth.make_graph(3, 20, 15, 24, k=260, depth=(5.5, 6.5), name="wall260")
    with pytest.raises(lm.LMError) as e:
        lm.solve_graph(g, elimination=lm.ELIM_CAPTURES)
    assert e.value.code == -2
    ref = oracle.solve_graph(g)
    ours = lm.solve_graph(g, elimination=lm.ELIM_AUTO)
    assert ours[3]["elimination_used"] == lm.ELIM_TAGS
    _compare_solves(g, ours, ref)
