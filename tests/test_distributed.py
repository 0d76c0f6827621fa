"""Capture-sharded LM across ranks (cfg4's decomposition) on CPU with gloo.

Each rank holds a contiguous capture range, its observations and every tag
(bench.shard_graph).  The per-step exchange -- the all-reduce of the reduced
tag+camera system and right-hand side, of the tag-side gradient / column
norms and of the scalar sums (cost, model cost change, step norm) -- is the
same decomposition the GPU path runs over RCCL.  Here it runs through the CPU
oracle's reduction hooks over torch.distributed gloo, world_size 2 and 3, and
must reproduce the single-process solve.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from ar_slam_amd import synth
        from oracle import oracle as O
        g = synth.config_graph(name)
        part = bench.shard_graph(g, rank, world)

        def s_fn(a):
            dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM)

        def m_fn(a):
            dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.MAX)

        comm = O.make_comm(rank, s_fn, m_fn)
        cam, cap, tag, s = O.solve(part["camera"], part["cap"], part["tag"], part["obs_cap"],
                                   part["obs_tag"], part["corners"], comm=comm)
        q.put((rank, cam, cap, tag, [it["cost"] for it in s["iterations"]], s["termination"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_oracle_matches_single_process(oracle, world):
    import multiprocessing as mp
    from ar_slam_amd import synth
    name = "small"
    g = synth.config_graph(name)
    cam0, cap0, tag0, s0 = oracle.solve_graph(g)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda t: t[0])
    costs0 = [it["cost"] for it in s0["iterations"]]
    for rank, cam, cap, tag, costs, term in res:
        assert term == s0["termination"]
        np.testing.assert_allclose(costs, costs0, rtol=1e-10)
        np.testing.assert_allclose(cam, cam0, rtol=1e-9)
        np.testing.assert_allclose(tag, tag0, rtol=1e-7, atol=1e-8)
    caps = np.concatenate([r[2] for r in res])
    np.testing.assert_allclose(caps, cap0, rtol=1e-7, atol=1e-8)


def test_shard_graph_partitions_captures():
    import bench
    from ar_slam_amd import synth
    g = synth.config_graph("medium")
    parts = [bench.shard_graph(g, r, 4) for r in range(4)]
    assert sum(p["cap"].shape[0] for p in parts) == g.n_cap
    assert sum(p["obs_cap"].shape[0] for p in parts) == g.n_obs
    for p in parts:
        assert p["obs_cap"].min() >= 0 and p["obs_cap"].max() < p["cap"].shape[0]
        assert p["tag"].shape == g.tag.shape
