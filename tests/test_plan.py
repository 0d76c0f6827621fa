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


@pytest.mark.parametrize("k", [600, 1000])
def test_mixed_set_layout_is_as_shallow_as_captures(L, k):
    """Ceres' mixed set on a cfg2 prefix (ELIM_MIXED): its reduced side holds tags and the
    captures next to eliminated tags, about as many rows as eliminating every capture.  The
    geometric separators place those captures at the mean of the tags they see -- at their own
    translation slot (minus the camera centre) the cuts were of a mirrored cloud and the tree
    grew taller (round 6: cfg2[:1000] 13 levels / 272 tiles against 11 / 205)."""
    g = synth.prefix_graph(synth.config_graph("cfg2"), k)
    args = (g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag)
    side_c, c = L.debug_reduced_plan_side(*args, elimination=L.ELIM_CAPTURES)
    side_m, m = L.debug_reduced_plan_side(*args, elimination=L.ELIM_MIXED)
    assert (side_c, side_m) == (L.ELIM_CAPTURES, L.ELIM_MIXED)
    assert c["dag_valid"] and m["dag_valid"]
    assert m["n_levels"] <= c["n_levels"] + 1
    assert m["n_factor_tiles"] <= 1.3 * c["n_factor_tiles"] * m["n_reduced"] / c["n_reduced"]


def test_invalid_problem_rejected_on_host(L):
    g = synth.config_graph("tiny")
    bad = g.obs_tag.copy()
    bad[0] = g.n_tag
    with pytest.raises(L.LMError):
        L.debug_reduced_plan(g.camera, g.cap, g.tag, g.obs_cap, bad, g.corners)


@pytest.mark.parametrize("name", ["medium", "cfg2", "cfg3"])
def test_task_graph_is_deadlock_free(L, name):
    """The persistent executor's ticket order: every wait is met by earlier tickets when run one at a
    time, and interleavings of 1..512 concurrent workgroups (the executor's 448 and the small-graph
    grid included), random and adversarial, never deadlock (dag_check / dag_simulate behind
    arslam_debug_reduced_plan)."""
    g = synth.config_graph(name)
    for ordering in (1, 2):
        info, _ = _plan(L, g, ordering=ordering)
        assert info["n_dag_tasks"] > 0
        assert info["dag_valid"] == 1, info
        # every fill tile's first application is an unfolded update item, so the solver may leave
        # the fill tiles uncleared (their first update stores 0 - acc); the plan checks it itself
        if info["n_factor_tiles"] > info["n_assembled_tiles"]:
            assert info["fill_first_ok"] == 1, info


def _brute_force_scalar_flops(g, tag_row, cam_rows=3):
    """Scalar Cholesky flops of the reduced system's real rows in the solver's order, by a
    column-by-column symbolic factorization: column j's below-diagonal structure is its own
    (tags co-visible in some capture, dense 6x6 blocks; the camera rows coupled to every
    tag) merged with the structures of the earlier columns whose first below-diagonal entry
    is j (the elimination-tree children).  Per column with c below-diagonal entries:
    c(c+1) + c + 1 flops (c divisions, c(c+1)/2 multiply-adds of the update, one sqrt)."""
    used = np.unique(g.obs_tag)
    order = sorted(used, key=lambda t: tag_row[t])                 # tags in reduced-row order
    pos = {t: i for i, t in enumerate(order)}
    n = 6 * len(order) + cam_rows
    struct = [set() for _ in range(n)]
    for c in range(g.n_cap):
        ts = sorted(pos[t] for t in g.obs_tag[g.obs_cap == c])
        for a in ts:
            for b in ts:
                if b > a:
                    for i in range(6):
                        struct[6 * a + i].update(range(6 * b, 6 * b + 6))
    for a in range(len(order)):                                    # inside a tag block, and to the camera
        for i in range(6):
            struct[6 * a + i].update(range(6 * a + i + 1, 6 * a + 6))
            struct[6 * a + i].update(range(6 * len(order), n))
    for k in range(6 * len(order), n):
        struct[k].update(range(k + 1, n))
    flops = 0.0
    for j in range(n):
        s = struct[j]
        c = len(s)
        flops += c * (c + 1) + c + 1
        if s:
            p = min(s)
            struct[p].update(x for x in s if x > p)
    return flops


@pytest.mark.parametrize("name", ["tiny", "small", "medium"])
def test_scalar_flops_match_symbolic_factorization(L, name):
    """summary.factor_scalar_flops (the roofline's algorithmic count) equals a brute-force
    symbolic Cholesky of the real rows in the same elimination order."""
    g = synth.config_graph(name)
    info, tag_row = _plan(L, g)
    assert info["scalar_flops"] == pytest.approx(_brute_force_scalar_flops(g, tag_row), rel=1e-12)


@pytest.mark.parametrize("name,worlds", [("medium", [2, 3]), ("cfg2", [2, 3, 4, 8]), ("cfg3", [2, 4, 8])])
def test_rank_split_partitions_the_factorization(L, name, worlds):
    """The multi-GPU split (arslam::rank_split, llt_plan_symbolic with column classes): every rank
    derives the same capture owners from the whole problem; the ranks' subtree columns and the
    replicated top columns partition the tile columns; each rank's two-phase task graph (its
    subtrees before the exchange, the top after it) is deadlock-free; and the exchange -- the
    top columns' tiles -- is a small part of the factor (cfg3 at 2 ranks: 55 of 2,461 tiles,
    where the replicated path all-reduced the 1,535 assembled ones)."""
    g = synth.config_graph(name)
    single, _ = _plan(L, g)
    for world in worlds:
        infos, owners = [], None
        for r in range(world):
            info, own = L.debug_rank_split(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, world, r)
            infos.append(info)
            if owners is None:
                owners = own
            np.testing.assert_array_equal(own, owners)
            assert info["dag_valid"] == 1, (world, r, info)
            assert 0 < info["phase_split"] <= info["n_dag_tasks"] or info["n_own_cols"] == 0
        assert owners.min() >= 0 and owners.max() < world
        assert [int((owners == r).sum()) for r in range(world)] == [i["n_owned_captures"] for i in infos]
        T = single["tiles_per_side"]
        assert infos[0]["n_top_cols"] + sum(i["n_own_cols"] for i in infos) == T
        assert all(i["n_top_tiles"] == infos[0]["n_top_tiles"] for i in infos)
        if name != "medium":   # (a 36-tile graph split 3 ways is mostly top)
            assert infos[0]["n_top_tiles"] < 0.5 * single["n_factor_tiles"]
    if name == "cfg3":
        info, _ = L.debug_rank_split(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, 2, 0)
        assert info["n_top_tiles"] <= 100 and info["n_top_tiles"] * 32768 < 4e6
        # the modelled split keeps the top small as N grows: ranks beyond the
        # useful subtree count stay idle in phase 0 instead of growing the exchange
        for world in (4, 8):
            info, owners = L.debug_rank_split(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, world, 0)
            assert info["n_top_tiles"] <= 100, (world, info)
            assert 2 <= info["n_active"] <= world


@pytest.mark.parametrize("name,cuts", [("small", [1, 17, 40]), ("cfg2", [300, 700, 999])])
def test_gather_plan_extension_equals_a_fresh_plan(L, name, cuts):
    """The appended-problem path (try_extend) extends the loaded Schur gather plan by the new
    captures' contributions instead of rebuilding it: every destination keeps its contributions in
    capture order (the gather's fixed summation order) and gains the new ones after them.  The
    result must be the fresh plan of the grown problem, array for array."""
    g = synth.config_graph(name)
    for c0 in cuts:
        same, nd = L.debug_gather_extend(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, c0)
        assert same, (name, c0)
        assert nd > 0


@pytest.mark.parametrize("name", ["small", "medium"])
def test_simulation_finds_the_deadlock_without_the_claim_cap(L, name):
    """The protocol simulation has teeth: a claimed continuation target may wait on tickets not yet
    drawn (its late waits), so without the cap on claimed targets in flight one workgroup claims a
    target and waits forever.  With the cap (the kernel's protocol) every policy finishes."""
    g = synth.config_graph(name)
    assert not L.debug_dag_simulate(g, 1, policy=1 + 16)
    for pol in range(4):
        assert L.debug_dag_simulate(g, 1, policy=pol)
        assert L.debug_dag_simulate(g, 2, seed=3, policy=pol)


def _fault_record_checks():
    from ar_slam_amd import lm as L
    g = synth.config_graph("cfg3")
    rec = [2772, 1, 340, 0, 1, 3000, 3, 17]
    s = L.debug_dag_fault_detail(g, rec)
    assert s.startswith("ticket 2772 (TRSM (80,69))"), s
    assert "ready[340] = 0 < 1" in s and "ticket 2205 (POTRF 69+TRSM) [continuation target]" in s, s
    assert "tickets drawn 3000" in s and "in flight 3" in s, s
    assert "smallest ticket timed out" not in s, s
    s3 = L.debug_dag_fault_detail(g, rec + [2**31 - 1 - 2205])   # a stuck chain starting at POTRF 69
    assert s3.endswith("smallest ticket timed out: 2205 (POTRF 69+TRSM)"), s3
    s2 = L.debug_dag_fault_detail(g, [2772, 1, 12625 * 0 + 2461 + 1620, 1, 2, 3000, 3, 17])
    assert "applied[1620] = 1 < 2" in s2 and "ticket 1981" in s2 and "ticket 2355" in s2, s2


def test_fault_record_names_the_stuck_counter_and_its_producers(L):
    """The record round 4's unexplained cfg3 fault would now carry (ticket 2772 timed out in its
    dependency wait): the message names the task, the counter, the value seen and the
    producers of the counter, with continuation targets marked -- here ticket 2772 = TRSM (80,69),
    waiting for L_69,69 from ticket 2205, a POTRF two predecessors may claim.  The record belongs to
    round 4's plan, i.e. to the dissection's height weight of then (ARSLAM_ND_BETA=0.6; the default
    is 0.3 since round 6), so the checks run in a process of their own under that weight."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ARSLAM_ND_BETA="0.6", PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    code = "import sys; sys.path.insert(0, %r); from tests.test_plan import _fault_record_checks as f; f()" % root
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]


@pytest.mark.parametrize("name", ["small", "medium", "cfg2"])
def test_claim_cap_follows_started_workgroups(L, name):
    """Progress independent of residency.  A 448-workgroup grid of which only
    k ever become resident: round 5's cap (half the grid) lets every resident workgroup hold a
    claimed continuation whose late waits name tickets nobody is left to draw -- the simulation
    finds that deadlock at k = 1; the kernel's cap (half the workgroups started so far) finishes
    every schedule at k = 1, 2, 7 and 64."""
    g = synth.config_graph(name)
    GRID_CAP = 32
    assert not any(L.debug_dag_simulate(g, 448, seed=1, policy=pol + GRID_CAP, started=1) for pol in range(4))
    for k in (1, 2, 7, 64):
        for pol in range(4):
            assert L.debug_dag_simulate(g, 448, seed=3, policy=pol, started=k), (k, pol)
