"""Debug the multi-rank path on one GPU: N worker processes (host-callback transport over
gloo), each logging its all-reduce calls and a faulthandler traceback to gpurun_out/mr_rank<r>.txt.
usage: python tools/mr_debug.py <config> <world>"""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, name):
    import numpy as np
    import torch
    import torch.distributed as dist
    log = open(os.path.join(ROOT, "gpurun_out", f"mr_rank{rank}.txt"), "w", buffering=1)
    faulthandler.dump_traceback_later(45, repeat=True, file=log)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ar_slam_amd import lm, synth
    g = synth.config_graph(name)
    ncall = [0]

    def allreduce(a, op):
        ncall[0] += 1
        print(f"{time.time():.3f} allreduce #{ncall[0]} n={a.size} {a.dtype} op={op}", file=log)
        dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)

    print("loading", file=log)
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners,
                            comm=(rank, world, allreduce), device=0)
    print("loaded; owned", len(rp.owned_captures()), file=log)
    s = rp.solve()
    print("solved", s["termination"], s["rule"], [it["cost"] for it in s["iterations"]], file=log)
    dist.destroy_process_group()


if __name__ == "__main__":
    import multiprocessing as mp
    name, world = sys.argv[1], int(sys.argv[2])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, world, port, name)) for r in range(world)]
    for p in ps:
        p.start()
    t0 = time.time()
    while any(p.is_alive() for p in ps) and time.time() - t0 < 100:
        time.sleep(5)
        print(f"{time.time() - t0:.0f}s alive {[p.is_alive() for p in ps]}", flush=True)
    for p in ps:
        if p.is_alive():
            p.kill()
    print("exit codes", [p.exitcode for p in ps], flush=True)
