"""Per-rank timing of the multi-GPU split with every rank alone on the GPU.

record: N ranks on one GPU (host-callback transport over gloo) solve the
        config once; each rank saves the result of every all-reduce it made
        (gpurun_out/replay_<cfg>_<N>_r<rank>.npz).
replay: one process per rank, alone on the GPU, loads the whole problem as
        that rank and solves with a transport that hands back the recorded
        results: the same numbers (so the same LM trace) with no other rank
        competing for the GPU -- the rank's own device time per phase.
model:  per LM iteration, the slowest rank's sharded work (linearize, Schur
        assembly, own-subtree factorization, back-substitution + cost) plus
        the replicated top factorization and backward solve, plus the
        exchange estimated from its bytes (ring all-reduce over xGMI).
usage: python tools/rank_replay.py record <cfg> <N> | replay <cfg> <N> | model <cfg> <N...>
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "gpurun_out")
REC = os.environ.get("TMPDIR", "/tmp")   # the recorded exchanges (large): not merged back
KEYS = ("t_linearize_ms", "t_schur_ms", "t_cholesky_ms", "t_factor_own_ms", "t_factor_top_ms",
        "t_solve_ms", "t_backsub_ms", "t_cost_ms")


def _rec_worker(rank, world, port, name):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ar_slam_amd import lm, synth
    g = synth.config_graph(name)
    rec = []

    def allreduce(a, op):
        dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
        rec.append(a.copy())

    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                            comm=(rank, world, allreduce), device=0)
    rec.clear()
    s = rp.solve()
    np.savez(os.path.join(REC, f"replay_{name}_{world}_r{rank}.npz"), *rec)
    with open(os.path.join(OUT, f"replay_{name}_{world}_r{rank}.json"), "w") as f:
        json.dump({"costs": [it["cost"] for it in s["iterations"]], "calls": len(rec)}, f)
    dist.destroy_process_group()


def record(name, world):
    import multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rec_worker, args=(r, world, port, name)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
    print("record", name, world, [p.exitcode for p in ps], flush=True)


def replay(name, world, solves=4):
    import numpy as np
    from ar_slam_amd import lm, synth
    g = synth.config_graph(name)
    rows = []
    for rank in range(world):
        if world == 1:
            rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, device=0, phase_timing=1)
        else:
            z = np.load(os.path.join(REC, f"replay_{name}_{world}_r{rank}.npz"))
            recs = [z[f"arr_{i}"] for i in range(len(z.files))]
            pos = [0]

            def allreduce(a, op, recs=recs, pos=pos):
                a[:] = recs[pos[0]]
                pos[0] += 1

            rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                                    comm=(rank, world, allreduce), device=0, phase_timing=1)
        acc = {k: 0.0 for k in KEYS}
        n_it = 0
        s = None
        for i in range(solves + 1):
            if world > 1:
                pos[0] = 0
            s = rp.solve()
            if i == 0:
                continue   # warm-up
            for k in KEYS:
                acc[k] += s[k]
            n_it += s["num_linear_solves"]
        row = {k: acc[k] / n_it for k in KEYS}
        row.update(rank=rank, iters=s["num_linear_solves"], owned=s["n_owned_captures"],
                   comm_mb_per_it=s["comm_bytes"] / s["num_linear_solves"] / 1e6, top_tiles=s["n_top_tiles"],
                   comm_calls_per_it=s["comm_calls"] / s["num_linear_solves"],
                   costs=[it["cost"] for it in s["iterations"]])
        rows.append(row)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items() if k != "costs"}),
              flush=True)
        rp.close()
    with open(os.path.join(OUT, f"replay_{name}_{world}.json"), "w") as f:
        json.dump(rows, f, indent=1)


def model(name, worlds, gbps=100.0, lat_us=25.0):
    """Predicted LM step per N from the per-rank replays (ms per LM iteration).

    Measured per rank alone on the GPU: the Schur assembly and the two factorization phases
    (no exchange inside their timers).  The linearization, back-substitution and cost timers
    of a replayed rank contain its host-staged exchanges (each a device->host copy, a sync and
    a copy back), so those per-capture kernels are taken from the one-rank run, scaled by the
    rank's share of the captures.  The exchange is estimated from its bytes."""
    out = []
    one = json.load(open(os.path.join(OUT, f"replay_{name}_1.json")))[0]
    per_cap = (one["t_linearize_ms"] + one["t_backsub_ms"] + one["t_cost_ms"]) / one["owned"]
    for world in worlds:
        rows = json.load(open(os.path.join(OUT, f"replay_{name}_{world}.json")))
        if world == 1:
            shard, top = one["t_linearize_ms"] + one["t_schur_ms"] + one["t_backsub_ms"] + one["t_cost_ms"], \
                one["t_cholesky_ms"]
            own = 0.0
        else:
            shard = max(per_cap * r["owned"] + r["t_schur_ms"] + r["t_factor_own_ms"] for r in rows)
            own = max(r["t_factor_own_ms"] for r in rows)
            top = rows[0]["t_factor_top_ms"]
        solve = one["t_solve_ms"]
        mb = rows[0]["comm_mb_per_it"] if world > 1 else 0.0
        calls = rows[0].get("comm_calls_per_it", 7.0) if world > 1 else 0.0   # (the solver's own count)
        # ring all-reduce: 2 (N-1)/N of the bytes over the link, plus a latency per collective
        exch = (2.0 * (world - 1) / world * mb * 1e6 / (gbps * 1e9) * 1e3 + calls * lat_us * 1e-3) if world > 1 else 0.0
        step = shard + top + solve + exch
        out.append({"n_gpus": world, "sharded_incl_own_factor_ms": shard, "own_factor_ms": own,
                    "top_or_full_factor_ms": top, "bsolve_ms": solve, "exchange_mb": mb,
                    "exchange_ms_est": exch, "collectives_per_iteration": calls, "step_ms": step})
    base = out[0]["step_ms"]
    for o in out:
        o["speedup_vs_1"] = base / o["step_ms"]
        print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in o.items()}))
    with open(os.path.join(OUT, f"replay_{name}_model.json"), "w") as f:
        json.dump({"assumptions": f"exchange = ring all-reduce at {gbps} GB/s algorithm bandwidth + {lat_us} us "
                                  "per collective (the solver's own count per LM iteration, summary.comm_calls); "
                                  "Schur assembly and both factorization "
                                  "phases measured per rank alone on one MI355X (tools/rank_replay.py); "
                                  "linearize/back-substitution/cost from the one-rank run scaled by owned captures",
                   "rows": out}, f, indent=1)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    mode, name = sys.argv[1], sys.argv[2]
    if mode == "record":
        record(name, int(sys.argv[3]))
    elif mode == "replay":
        replay(name, int(sys.argv[3]))
    else:
        model(name, [int(a) for a in sys.argv[3:]])
