"""Capture-sharded GPU solve across ranks (cfg4's decomposition), on one GPU.

Two processes share cuda:0 (RCCL needs one GPU per rank, so the exchange runs
through arslam_lm_set_comm_callback over torch.distributed gloo).  Every
exchange the RCCL path makes -- tag degrees, the co-visibility pattern, the
Jacobi column norms, the assembled prefix of the reduced system with its
rhs, the LM scalar sums -- goes through the same solver code; only the
transport differs.  The sharded solve must reproduce the single-process
oracle (tolerances as tests/test_gpu_parity.py) and give the same trace on
every rank.

The parent process never touches the GPU itself (it checks the device count
with torch.cuda.device_count(), which does not initialise HIP here), so
spawning the workers is a plain child-process start.
"""
import os
import socket

import numpy as np
import pytest

from gauge import assert_poses_match, load_cfg3_golden

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, q, abort_rank=-1):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ar_slam_amd import lm, synth
        g = synth.config_graph(name)
        part = dict(camera=g.camera, cap=g.cap, tag=g.tag, obs_cap=g.obs_cap, obs_tag=g.obs_tag,
                    corners=g.corners)   # every rank loads the whole problem

        def allreduce(a, op):
            dist.all_reduce(torch.from_numpy(a),
                            op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)

        rp = lm.ResidentProblem(**part, comm=(rank, world, allreduce), device=0)
        if abort_rank >= 0:   # only this rank's callback asks to stop, at iteration 2
            rp.set_iteration_callback(
                lambda it: lm.SOLVER_ABORT if rank == abort_rank and it["iteration"] == 2 else None)
        s = rp.solve()
        own = rp.owned_captures()
        q.put((rank, rp.camera.copy(), (own, rp.cap[own].copy()), rp.tag.copy(),
               [it["cost"] for it in s["iterations"]], s["termination"], s["rule"], s["final_cost"],
               s["comm_bytes"] / max(s["num_linear_solves"], 1),
               [it["trust_region_radius"] for it in s["iterations"]], s["n_top_tiles"],
               (s["comm_calls"], s["num_linear_solves"])))
    except Exception as e:   # noqa: BLE001 -- surface the failure in the parent
        q.put((rank, None, None, None, None, repr(e), None, None, None, None, None, None))
    finally:
        dist.destroy_process_group()


def _run_ranks(name, world, abort_rank=-1):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q, abort_rank)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    res.sort(key=lambda t: t[0])
    for r in res:
        assert r[1] is not None, r[5]
    return res


def _gather_caps(res, n_cap):
    """The captures' final poses from their owning ranks (every capture owned exactly once)."""
    cap = np.full((n_cap, 6), np.nan)
    seen = np.zeros(n_cap, int)
    for r in res:
        own, poses = r[2]
        cap[own] = poses
        seen[own] += 1
    assert np.all(seen == 1), "every capture is owned by exactly one rank"
    return cap


def _same_on_every_rank(res):
    """The exchanged sums are identical on every rank: the same trace, camera and tags."""
    for r in res[1:]:
        assert r[4] == res[0][4]
        np.testing.assert_array_equal(r[1], res[0][1])
        np.testing.assert_array_equal(r[3], res[0][3])


@pytest.mark.parametrize("name,world", [("medium", 2), ("cfg2", 2), ("cfg2", 3), ("cfg2", 4), ("kvar", 2),
                                        ("k24", 2)])
def test_sharded_gpu_solve_matches_oracle(oracle, name, world):
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    from ar_slam_amd import synth
    g = synth.config_graph(name)
    cam0, cap0, tag0, s0 = oracle.solve_graph(g)
    res = _run_ranks(name, world)
    costs0 = [it["cost"] for it in s0["iterations"]]
    _same_on_every_rank(res)
    rank, cam, _, tag, costs, term, rule, final = res[0][:8]
    assert term == s0["termination"] and rule == s0["rule"]
    assert abs(len(costs) - len(costs0)) <= 1
    for a, b in list(zip(costs, costs0))[:5]:
        assert abs(a - b) <= 1e-9 * abs(b)
    assert abs(final - s0["final_cost"]) <= 1e-8 * s0["final_cost"]
    assert abs(cam[0] - cam0[0]) <= 1e-8 * cam0[0]
    # the captures, each from its owner, and the tags, in the oracle's gauge (aligned by the tags)
    cap = _gather_caps(res, g.n_cap)
    assert_poses_match(cap, tag, cap0, tag0, tags=np.unique(g.obs_tag))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_cfg3_matches_golden_trace(world):
    """cfg4's decomposition at the headline size: cfg3 (10k captures / 2k tags) split over 2, 4 and
    8 ranks (the subtree-to-rank split of the reduced system's elimination tree; every exchange
    through the host callback, all ranks on one GPU), against the oracle's committed cfg3 trace
    (tests/golden/lm_cfg3.json).  The exchange per LM iteration is the top columns' tiles (a few
    MB; all-reducing the assembled reduced system was 50.5 MB) plus y and the LM scalars."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    import json
    from ar_slam_amd import synth
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lm_cfg3.json")) as f:
        gold = json.load(f)
    res = _run_ranks("cfg3", world)
    _same_on_every_rank(res)
    rank, cam, _, tag, costs, term, rule, final, xbytes, radius, top_tiles, (calls, solves) = res[0]
    assert (term, rule) == (gold["termination"], gold["rule"])
    assert abs(len(costs) - len(gold["cost"])) <= 1
    for a, b in list(zip(costs, gold["cost"]))[:5]:
        assert abs(a - b) <= 1e-9 * abs(b), (costs, gold["cost"])
    np.testing.assert_allclose(radius[:5], gold["trust_region_radius"][:5], rtol=1e-12)
    assert abs(final - gold["final_cost"]) <= 1e-8 * gold["final_cost"]
    assert abs(cam[0] - gold["final_focal"]) <= 1e-8 * gold["final_focal"]
    g = synth.config_graph("cfg3")
    _, fin = load_cfg3_golden()
    e = assert_poses_match(_gather_caps(res, g.n_cap), tag, fin["cap"], fin["tag"])
    print(f"cfg3 x{world} pose errors vs the oracle: {e}")
    print(f"cfg3 x{world} ranks: {xbytes / 1e6:.1f} MB all-reduced per rank per LM iteration "
          f"({top_tiles} top tiles)")
    assert xbytes <= top_tiles * 32768 + 1e6 and xbytes < 20e6
    # collectives per LM iteration: two -- the top tiles (with an accepted step's linearization's tag
    # sums in front of them) and the step's scalars (with that linearization's cost and norms); +
    # iteration 0's two, a stop before a step's two, and the final tag gather
    print(f"cfg3 x{world}: {calls} collectives over {solves} LM iterations")
    assert calls <= 2 * solves + 5, (calls, solves)


def test_iteration_callback_decision_is_agreed_across_ranks():
    """One rank's iteration callback returns SOLVER_ABORT at iteration 2, the other's CONTINUE:
    the ranks take the same branch (the callbacks' answers are MAX-all-reduced), so every rank
    ends with USER_FAILURE after the same three recorded iterations instead of one rank leaving
    while the other blocks in the next step's exchange."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    res = _run_ranks("medium", 2, abort_rank=1)
    for r in res:
        assert (r[5], r[6]) == ("USER_FAILURE", "user_callback"), r[5:7]
        assert len(r[4]) == 3 and r[4] == res[0][4]


def test_bench_launches_its_ranks():
    """`bench.py --gpus 2` with no launcher environment starts its two rank processes itself and emits
    ONE line for the job: n_gpus 2, the split over 2 ranks with its active-rank count.  The exchange
    runs through the host callback over gloo with both ranks on the one GPU of this box (the
    driver's multi-GPU runs use RCCL, one GPU per rank)."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--config", "medium",
                          "--transport", "callback", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                          "--no-incremental", "--no-localize", "--no-fingerprint"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["split"]["n_ranks"] == 2 and 1 <= d["split"]["active_ranks"] <= 2, d["split"]
    assert d["value"] > 0 and d["termination"].startswith("CONVERGENCE"), d
    assert "callback" in d["transport"], d["transport"]


def _one_rank_worker(name, q):
    """One process: the plain one-rank solve, then the forced multi-rank path on one rank through
    the host callback (identity all-reduce) and through a one-rank RCCL communicator."""
    try:
        from ar_slam_amd import lm, synth
        g = synth.config_graph(name)
        part = dict(camera=g.camera, cap=g.cap, tag=g.tag, obs_cap=g.obs_cap, obs_tag=g.obs_tag,
                    corners=g.corners)
        out = {}
        for mode in ("plain", "callback", "rccl"):
            comm = None
            if mode == "callback":
                comm = (0, 1, lambda a, op: None)   # one rank: the all-reduce is the identity
            elif mode == "rccl":
                comm = (0, 1, lm.comm_unique_id())
            rp = lm.ResidentProblem(**part, comm=comm, force_multirank=mode != "plain", device=0)
            s = rp.solve()
            out[mode] = (rp.camera.copy(), rp.cap.copy(), rp.tag.copy(), [it["cost"] for it in s["iterations"]],
                         [it["trust_region_radius"] for it in s["iterations"]], s["termination"], s["rule"],
                         s["comm_calls"], s["comm_bytes"], s["n_top_tiles"], s["n_ranks"])
            rp.close()
        q.put(out)
    except Exception as e:   # noqa: BLE001 -- surface the failure in the parent
        q.put(repr(e))


def test_one_rank_rccl_path_runs_the_real_collectives():
    """RCCL on hardware with one GPU: arslam_lm_debug_force_multirank makes the
    handle take the multi-rank path with one rank -- the two-rank split's replicated top, the
    two-phase factorization, the top-tile all-reduce, the all-gathered step scalars, the u8 MAX
    flags, the split-hash check and the final tag gather -- and arslam_lm_set_comm(0, 1, id) then
    runs ncclCommInitRank(nranks = 1) and every ncclAllReduce on the solver's stream.  A one-rank
    all-reduce is the identity, so the RCCL solve is bit-identical to the same path through the host
    callback; both agree with the plain one-rank solve to rounding (the two-phase factorization sums
    a top tile's updates subtree-first, so the last bits may differ) and match it pose for pose."""
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank_worker, args=("cfg2", q))
    p.start()
    try:
        out = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert isinstance(out, dict), out
    plain, cb, rc = out["plain"], out["callback"], out["rccl"]
    # the transport is all that differs: bit-identical
    for a, b in zip(cb[:5], rc[:5]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    assert cb[5:] == rc[5:]
    calls, xbytes, top_tiles, nr = rc[7:]
    assert nr == 1 and calls > 0 and top_tiles > 0 and xbytes >= top_tiles * 32768, rc[7:]
    assert plain[7] == 0   # the plain path makes no collective
    # the multi-rank path on one rank against the plain solve
    assert (rc[5], rc[6]) == (plain[5], plain[6])
    assert len(rc[3]) == len(plain[3])
    for a, b in zip(rc[3], plain[3]):
        assert abs(a - b) <= 1e-9 * abs(b), (rc[3], plain[3])
    np.testing.assert_allclose(rc[4], plain[4], rtol=1e-9)
    assert abs(rc[0][0] - plain[0][0]) <= 1e-8 * plain[0][0]
    assert_poses_match(rc[1], rc[2], plain[1], plain[2])
    same = all(np.array_equal(np.asarray(a), np.asarray(b)) for a, b in zip(rc[:4], plain[:4]))
    print(f"one-rank RCCL path: {calls} collectives, {xbytes / 1e6:.2f} MB, {top_tiles} top tiles; "
          f"bit-identical to the plain solve: {same}")
