#!/usr/bin/env python3
"""Benchmark of the MI355X LM bundle adjuster on BASELINE.json's headline workload.

Metric (BASELINE.json): "LM iterations/sec + ms-to-converged reproj-RMS,
10k-capture synthetic graph".  One *step* is one complete ceres::Solve
equivalent (ar_slam_util.cpp:1001-1018) of cfg3 -- 10,000 captures, 2,000
tags, k = 8 observations per capture (80,000 residual blocks), seed 2 --
from the same initial state to the Ceres termination rule.  The problem is
uploaded to HBM before the timed region; every solve restarts from the
resident initial state.

  value        = LM iterations (trust-region step computations) of the K
                 timed solves / wall time of the K solves (max over ranks)
  ms_per_step  = ms-to-converged of one solve

Multi-GPU, one process per GPU: `python bench.py --gpus N` starts the N rank
processes itself (before anything touches the GPU; 127.0.0.1 rendezvous), or
run it under torchrun (`python -m torch.distributed.run --nnodes=1
--nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N`),
which sets WORLD_SIZE.  Every rank loads the whole problem and the solver
splits the reduced system's elimination tree below its top separators; each
rank factors its own subtrees (and owns their captures), then the top
columns' tiles are summed over RCCL and factored on every rank (the path has
a real exchange step, and total work is fixed: strong scaling).
`--transport callback` runs the same exchange through the host all-reduce
callback over gloo, every rank on the one GPU there is (a test transport: it
checks the multi-rank path end to end on a 1-GPU box, it measures no scaling).

The JSON line also carries the dominant kernel's roofline (the MFMA fp64
trailing update of the reduced-system Cholesky, timed with HIP events around
each of its launches inside the timed region) and a CPU baseline: the CPU
oracle (oracle/, a C port of the same algorithm, NOT Ceres) timed on a
bounded sample of the same workload on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "LM iterations/sec + ms-to-converged reproj-RMS, 10k-capture synthetic graph"
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X datasheet fp64 matrix (no f64 row in MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def shard_graph(g, rank, world):
    """Contiguous capture range of this rank; all tags replicated (the CPU oracle's sharded
    restatement, tests/test_distributed.py; the GPU path splits the whole problem itself)."""
    lo = (g.n_cap * rank) // world
    hi = (g.n_cap * (rank + 1)) // world
    sel = (g.obs_cap >= lo) & (g.obs_cap < hi)
    return dict(camera=g.camera, cap=g.cap[lo:hi], tag=g.tag,
                obs_cap=(g.obs_cap[sel] - lo).astype(np.int32), obs_tag=g.obs_tag[sel],
                corners=g.corners[sel])


def cpu_baseline(g, threads, name):
    """CPU oracle (the same algorithm as Ceres' DENSE_SCHUR + Eigen LLT, restated in C, NOT Ceres):
    one full solve of the workload to the Ceres termination rule."""
    from oracle import oracle as O
    O.build()
    t0 = time.perf_counter()
    _, _, _, s = O.solve_graph(g, num_threads=threads)
    dt = time.perf_counter() - t0
    iters = s["num_linear_solves"]
    return {"value": iters / dt, "unit": "LM iterations/s", "cores": threads, "kind": "port",
            "ms_to_converged": 1e3 * dt, "termination": f"{s['termination']} ({s['rule']})",
            "sample": f"one full {name} solve to termination ({iters} LM iterations, iteration-0 "
                      f"linearization included), CPU oracle (C, OpenMP dense LLT on {threads} threads), "
                      f"{dt:.1f} s"}


def bench_incremental(name="cfg2", elimination=0):
    """The reference's real flow (ArSlamSolver::solveIncremental, ar_slam_util.cpp:629-742): one
    Detections message per capture, each followed by a full Solve of the problem so far (:736),
    through the C++ host mirror and the pointer-keyed C-ABI (the drop-in path, host buffers, setup
    included).  Reported beside the headline line, never as `value`."""
    from ar_slam_amd import lm, synth
    g = synth.config_graph(name)
    s = lm.SlamSolver(elimination=elimination)   # (0: the mirror's default, Ceres' exact set)
    s.set_camera(g.camera)
    t0 = time.perf_counter()
    for c in range(g.n_cap):
        sel = g.obs_cap == c
        s.add_detections(f"cap{c}", [f"tag_{t}" for t in g.obs_tag[sel]], g.corners[sel])
        s.solve_incremental()
    wall = time.perf_counter() - t0
    n = s.num_solves
    sums = [s.solve_summary(i) for i in range(n)]
    setup = sum(d["setup_time_s"] for d in sums)
    kinds = [sum(d["setup_kind"] == k for d in sums) for k in range(3)]
    mini = sum(d["minimizer_time_s"] for d in sums)
    return {"flow": f"solveIncremental on {name} ({g.n_cap} captures / {g.n_tag} tags), one message per capture",
            "wall_s": wall, "solves": n, "lm_iterations": sum(d["num_linear_solves"] for d in sums),
            "setup_ms_per_solve": 1e3 * setup / n, "minimizer_ms_per_solve": 1e3 * mini / n,
            "setup_kinds": {"full load": kinds[0], "values only": kinds[1], "appended (plan kept)": kinds[2]},
            # (the mirror's default: Ceres' own e-block set, ARSLAM_ELIM_MIXED -- all tags, then mixed)
            "elimination_used": {name: sum(d["elimination_used"] == e for d in sums)
                                 for e, name in ((lm.ELIM_CAPTURES, "captures"), (lm.ELIM_TAGS, "tags"),
                                                 (lm.ELIM_MIXED, "mixed"))},
            "final_rms_px": sums[-1]["final_rms_px"]}


def cgroup_cpu_quota():
    """The cgroup's CPU bandwidth limit in CPUs (cgroup v2 cpu.max "quota period", or v1's
    cfs_quota_us / cfs_period_us), with the raw text; None where there is no limit file."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                raw = f.read().strip()
        except OSError:
            continue
        if parse:
            q, p = (parse(raw) + ["100000"])[:2]
        else:
            q = raw
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    p = f.read().strip()
            except OSError:
                p = "100000"
        cpus = None if q in ("max", "-1") else int(q) / int(p)
        return {"file": path, "raw": raw, "cpus": cpus}
    return None


def host_cpu_info():
    """The CPUs this process may run on (the box's cpuset: one GPU's share of the node), the
    cgroup's CPU quota, and the node's own lscpu summary."""
    import subprocess
    info = {"nproc": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_quota": cgroup_cpu_quota()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keep = ("Model name", "CPU(s)", "Thread(s) per core", "Core(s) per socket", "Socket(s)")
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keep:
                info["lscpu_" + k.strip().lower().replace("(s)", "s").replace(" ", "_")] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def bench_localize(args, world, rank, side=False):
    """cfg5: batched localizeMany of 4096 queries against cfg3's map (BASELINE.json configs[4]).

    One step = one solve of the whole batch (every query's independent LM to
    its own termination) from the resident initial state.  Reported as
    queries/s; the per-query-iteration rate and the kernel's HBM roofline
    (algorithmic bytes: per query-iteration 2 passes over the observation
    records (72 B each) and the tag poses they gather (48 B each), plus the
    pose) ride along."""
    from ar_slam_amd import lm, synth
    import torch
    b = synth.make_localize_batch(n_query=4096)
    loc = lm.Localizer(b, device=0 if world == 1 else int(os.environ.get("LOCAL_RANK", "0")))
    _, res, _ = loc.solve()
    for _ in range(args.warmup):
        loc.solve(download=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = 0.0
    for _ in range(args.steps):
        _, _, ms = loc.solve(download=False)
        kms += ms
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:   # replicas: every rank localizes its own batch; the job is the slowest rank
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    q_iters = int(res["num_iterations"].sum())
    k_obs = b.n_obs / b.n_query
    bytes_per_qi = 2 * k_obs * (72 + 48) + 48
    avg_kernel_s = kms / args.steps * 1e-3
    # The kernel is bound by fp64 VALU issue (trig, divisions, DPP reductions),
    # not HBM: its roofline is VALU wave-instructions per second against one
    # instruction per 4 cycles per SIMD (a wave64 fp64 FMA; MI355X: 256 CUs x 4
    # SIMDs x 2.4 GHz), with the instruction count per launch from the
    # committed PMC pass (profiles/pmc_localize.json, SQ_INSTS_VALU).
    valu = load_pmc_localize()
    valu_peak = 256 * 4 * 2.4e9 / 4 / 1e9   # G wave-instructions/s
    achieved_valu = valu / avg_kernel_s / 1e9 if valu else None
    achieved = bytes_per_qi * q_iters / avg_kernel_s / 1e9
    out = {"metric": "localize queries/s, 4096-query batch against the 2k-tag cfg3 map",
           "value": world * b.n_query * args.steps / elapsed, "unit": "queries/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (seeded generator, SURVEY.md §8d cfg5)",
           "config": {"workload": f"cfg5: {b.n_query} queries x {int(k_obs)} tags, map = cfg3 tags",
                      "parallelism": "two queries per wavefront (32 lanes each)"},
           "query_iterations_per_s": world * q_iters * args.steps / elapsed,
           "mean_iterations_per_query": q_iters / b.n_query,
           "roofline": {"bound": "valu", "kernel": "k_localize (two queries per wave)",
                        "achieved": achieved_valu, "peak": valu_peak, "unit": "G VALU-instructions/s",
                        "frac": achieved_valu / valu_peak if achieved_valu else None,
                        "traffic": load_pmc_traffic("k_localize<2, 32>"), "traffic_source": PMC_PROFILE,
                        "avg_launch_us": avg_kernel_s * 1e6, "valu_instructions_per_launch": valu,
                        "hbm_view": {"achieved_GBps": achieved, "peak_GBps": HBM_PEAK_GBS,
                                     "frac": achieved / HBM_PEAK_GBS,
                                     "bytes_per_query_iteration": bytes_per_qi}},
           "cpu_baseline": None}
    if not args.no_cpu_baseline and world == 1:
        # (as the side key of the default line: a 4 s sample, so the line stays within minutes)
        from oracle import oracle as O
        O.build()
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < (4.0 if side else 10.0):
            O.localize_many(b)
            n += b.n_query
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": n / dt, "unit": "queries/s", "cores": 1, "kind": "port",
                               "sample": f"{n} queries (the cfg5 batch repeated) through the CPU oracle's "
                                         f"localizeMany, single thread, {dt:.1f} s"}
    if side:
        return out
    if rank == 0:
        print(json.dumps(out), flush=True)


def load_pmc_localize():
    """SQ_INSTS_VALU per k_localize launch from the committed PMC pass, if any."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_localize.json")) as f:
            return json.load(f).get("valu_instructions_per_launch")
    except (OSError, ValueError):
        return None


# the PMC passes of the commit this bench line measures (each profile round writes its own
# directory; these name the latest): HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md,
# tools/pmc_bench.sh) and the dominant kernel's MFMA utilisation (tools/pmc_mfma.sh)
PMC_PROFILE = os.path.join("profiles", "r06", "pmc_hbm_bytes.json")
PMC_MFMA = os.path.join("profiles", "r06", "pmc_mfma.json")


def _load_json(rel):
    try:
        with open(os.path.join(ROOT, rel)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def load_pmc_traffic(kernel="k_factor_dag"):
    """Per-launch HBM bytes of a kernel from the latest committed PMC pass, if any."""
    d = _load_json(PMC_PROFILE)
    try:
        return d["kernels"][kernel]["hbm_bytes_per_launch"]
    except (KeyError, TypeError):
        return None


def load_pmc_mfma():
    """k_factor_dag's MFMA busy fraction and issued fp64 MFMA flops from the latest PMC pass."""
    d = _load_json(PMC_MFMA)
    if not d:
        return {}
    return {k: d.get(k) for k in ("mfma_busy_frac", "mfma_busy_frac_at_2p4ghz", "effective_clock_ghz",
                                  "mfma_f64_flops_per_launch", "mfma_f64_tflops", "mean_us")}


def compulsory_factor_bytes(n_factor_tiles, n_reduced):
    """The least HBM traffic of one factorization: every factor tile read once (as assembled) and
    written once (as L), and each tile column's L_kk, L_kk^{-1} (64x64) and its four 16x16 block
    inverses written once -- no operand re-reads at all."""
    T = -(-(int(n_reduced) + 1) // 64)
    tile = 64 * 64 * 8
    return 2 * int(n_factor_tiles) * tile + T * (2 * tile + 4 * 16 * 18 * 8)


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` without a launcher: build first (CPU only), then start N rank processes of this
    script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each), forward rank 0's line and
    return the worst exit status.  This process never touches the GPU, so the children are plain
    child processes (no exec from a process that initialised HIP)."""
    import subprocess
    if not args.launch_check:
        from ar_slam_amd import build
        build.build()
    import tempfile
    import time
    port = _free_port()
    procs = []
    # rank 0's line goes to a file (no pipe to drain while the ranks are polled)
    out0 = tempfile.TemporaryFile()
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else sys.stderr, cwd=ROOT))
    # Poll every rank: a rank that dies (a bad build, an init error before the
    # rendezvous) would leave the others waiting in a collective forever, so
    # the first non-zero exit ends the rest and is returned.
    bad = 0
    while [p.poll() for p in procs].count(None):   # (every rank polled: no short-circuit)
        failed = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if failed:
            bad = failed[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.2)
    rcs = [p.wait() for p in procs]
    out0.seek(0)
    sys.stdout.write(out0.read().decode())
    sys.stdout.flush()
    if not bad:
        nz = [rc for rc in rcs if rc != 0]
        bad = nz[0] if nz else 0
    return bad


def launch_check(world, rank):
    """`--launch-check` (CPU, no GPU): the ranks meet over gloo and rank 0 prints who came -- the
    launcher and rendezvous of the multi-rank bench without a solve (tests/test_bench_launch.py)."""
    if os.environ.get("ARSLAM_LAUNCH_CHECK_FAIL_RANK") == str(rank):   # (test: a rank dying before the rendezvous)
        sys.exit(3)
    import torch
    import torch.distributed as dist
    t = torch.zeros(world, dtype=torch.int64)
    t[rank] = rank + 1
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "world_size": world,
                          "ranks": [int(v) - 1 for v in t.tolist()],
                          "env": {k: os.environ.get(k) for k in ("MASTER_ADDR", "LOCAL_WORLD_SIZE")}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-incremental", action="store_true", help="skip the solveIncremental (cfg2) side line")
    ap.add_argument("--no-localize", action="store_true", help="skip the cfg5 batched-localize side key")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--rccl-one-rank", action="store_true",
                    help="(debug, one GPU) the multi-rank path with one rank over a one-rank RCCL communicator "
                         "made through torch.distributed's nccl group: every collective of a multi-rank solve runs")
    ap.add_argument("--transport", choices=("rccl", "callback"), default="rccl",
                    help="multi-rank exchange: RCCL (one GPU per rank) or the host all-reduce callback over gloo "
                         "(test transport: every rank on the one GPU there is)")
    ap.add_argument("--launch-check", action="store_true",
                    help="(tests) start the ranks and meet over gloo, no GPU, no solve")
    ap.add_argument("--no-fingerprint", action="store_true", help="skip the in-process box fingerprint")
    ap.add_argument("--skip-zero-tiles", type=int, default=1)
    ap.add_argument("--ordering", type=int, default=2, help="0 natural, 1 RCM, 2 nested dissection")
    ap.add_argument("--executor", type=int, default=1, help="0 level launches, 1 persistent task graph")
    ap.add_argument("--no-runtime-warmup", action="store_true",
                    help="no small solve before the setup (profiling passes: rocprof's per-kernel averages then hold "
                         "only this workload's launches; the setup then includes the runtime start)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: measuring {world} ranks", file=sys.stderr)
    if args.launch_check:
        launch_check(world, rank)
        return
    # build (if stale) before anything touches the GPU; ranks serialize on the build lock
    from ar_slam_amd import build
    build.build()
    import torch
    import torch.distributed as dist
    callback = world > 1 and args.transport == "callback"
    device = local_rank
    if callback:   # every rank on the one GPU there is (device_count does not initialise HIP here)
        device = local_rank % max(1, torch.cuda.device_count())
        dist.init_process_group("gloo", rank=rank, world_size=world)
    elif world > 1 or args.rccl_one_rank:
        torch.cuda.set_device(local_rank)
        if world == 1:   # (--rccl-one-rank: a one-rank group, the same init and broadcast as N ranks)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if args.config == "cfg5":
        bench_localize(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    from ar_slam_amd import lm, synth
    g = synth.config_graph(args.config)
    # every rank loads the whole problem; the solver splits it (subtree-to-rank split of the
    # reduced system's elimination tree: each rank owns the captures of its subtrees)
    part = dict(camera=g.camera, cap=g.cap, tag=g.tag, obs_cap=g.obs_cap, obs_tag=g.obs_tag, corners=g.corners)
    comm = None
    if callback:
        def allreduce(a, op):
            dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
        comm = (rank, world, allreduce)
    elif world > 1 or args.rccl_one_rank:
        obj = [lm.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm = (rank, world, obj[0])
    opts = dict(device=device, kernel_timing=0 if args.no_kernel_timing else 1,
                cholesky_skip_zero_tiles=args.skip_zero_tiles, reduced_ordering=args.ordering,
                factor_executor=args.executor)
    # the timed solves record no per-phase events (each costs GPU time between
    # kernels); the dominant kernel's own events stay on for the roofline.
    # Construction = the cold per-problem setup a Ceres Solve's preprocessor
    # stands for: host structure, nested dissection, tile plan + task graph,
    # Schur gather plan, upload.
    # The process's one-time runtime start (the library's code objects loaded
    # on first launch, its stream and page-locked buffers) is paid by a small
    # solve first and reported on its own (runtime_init_s): a SLAM node pays it
    # once, every problem after it pays the setup below
    torch.cuda.set_device(device)
    torch.cuda.synchronize()
    runtime_init_s = None if args.no_runtime_warmup else lm.warm_up(device)
    torch.cuda.synchronize()
    t_setup = time.perf_counter()
    rp = lm.ResidentProblem(**part, comm=comm, phase_timing=0, force_multirank=args.rccl_one_rank, **opts)
    setup_wall_s = time.perf_counter() - t_setup

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        rp.solve()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sums = []
    for _ in range(args.steps):
        sums.append(rp.solve())
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if callback else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    iters = sum(s["num_linear_solves"] for s in sums)
    last = sums[-1]
    # one more solve, untimed, with the per-phase events on: the phase breakdown
    rp.set_options(phase_timing=1, **opts)
    phased = rp.solve()
    dom_ms = sum(s["t_dominant_ms"] for s in sums)
    dom_launches = sum(s["n_dominant_launches"] for s in sums)
    dom_flops = sum(s["dominant_flops"] for s in sums)
    roofline = None
    if dom_launches:
        avg_ms = dom_ms / dom_launches
        flops_per_launch = dom_flops / dom_launches          # the tile plan's flops (padding, zeros in fill tiles)
        scalar_flops = last["factor_scalar_flops"]          # scalar Cholesky of the real rows: the algorithmic count
        achieved = scalar_flops / (avg_ms * 1e-3) / 1e12
        achieved_tile = flops_per_launch / (avg_ms * 1e-3) / 1e12
        kname = ("k_factor_dag (reduced-system Cholesky, persistent task graph: POTRF + TRSM + "
                 "trailing updates on v_mfma_f64_16x16x4_f64)") if args.executor == 1 else \
            "k_update (reduced-system Cholesky trailing update, v_mfma_f64_16x16x4_f64)"
        traffic = load_pmc_traffic("k_factor_dag" if args.executor == 1 else "k_update")
        compulsory = compulsory_factor_bytes(last["n_factor_tiles"], last["n_reduced"])
        mf = load_pmc_mfma() if args.executor == 1 else {}
        roofline = {"bound": "mfma", "kernel": kname,
                    "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": traffic,
                    "traffic_source": PMC_PROFILE,
                    # PMC bytes / the least traffic of the factorization (every tile read and
                    # written once): > 1 is operand re-reads and the level-ordered target updates
                    "compulsory_bytes": compulsory,
                    "traffic_ratio": traffic / compulsory if traffic else None,
                    "mfma_busy_frac": mf.get("mfma_busy_frac"),
                    "mfma_counters": dict(mf, source=PMC_MFMA) if mf else None,
                    "avg_launch_us": avg_ms * 1e3,
                    "flops_per_launch": scalar_flops,
                    "flops_basis": "scalar Cholesky of the reduced system's real rows in the chosen order "
                                   "(sum over columns of c(c+1)+c+1; no padding rows, no zeros inside fill tiles)",
                    "tile_flops_per_launch": flops_per_launch,
                    "achieved_tile_flops": achieved_tile,
                    "frac_tile_flops": achieved_tile / FP64_MFMA_PEAK_TFLOPS,
                    # Ceres' DenseSchur factors the same real rows densely (Eigen LLT): n^3/3
                    "dense_llt_flops_equivalent": (6.0 * len(np.unique(g.obs_tag)) + 3.0) ** 3 / 3.0,
                    "launches": dom_launches}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": iters / elapsed,
            "unit": "LM iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded generator, SURVEY.md §8d)",
            "config": {"workload": f"{args.config}: {g.n_cap} captures / {g.n_tag} tags / "
                                   f"{g.n_obs} observations (k=8), one full LM solve per step",
                       "n_obs": int(g.n_obs), "n_reduced": int(last["n_reduced"]),
                       "parallelism": (f"subtree split x{world} ("
                                       + ("host-callback" if callback else "RCCL") + " all-reduce of the top tiles)")
                                      if world > 1 else "single GPU"},
            "ms_to_converged": 1e3 * elapsed / args.steps,
            # the cold setup of the problem (first load: ordering, plan, upload), outside the timed
            # region, and the ms-to-converged a first Solve of a new problem would see
            "setup_time_s": setup_wall_s,
            "setup_time_s_solver": last["setup_time_s"],
            "setup_phases_s": dict(zip(("structure", "elimination_order", "tile_plan", "gather_plan_and_upload",
                                        "other"), last["setup_phase_s"])),
            "runtime_init_s": runtime_init_s,
            "ms_to_converged_incl_setup": 1e3 * (elapsed / args.steps + setup_wall_s),
            "final_rms_px": last["final_rms_px"],
            "termination": f"{last['termination']} ({last['rule']})",
            "lm_iterations_per_solve": last["num_linear_solves"],
            "reduced_system": {"rows": int(last["n_reduced"]), "factor_tiles": int(last["n_factor_tiles"]),
                               "etree_levels": int(last["n_levels"]),
                               "ordering": ["natural", "RCM", "nested dissection"][args.ordering],
                               "executor": ["level launches", "persistent task graph"][args.executor],
                               "skip_zero_tiles": bool(args.skip_zero_tiles)},
            "comm_mb_per_lm_iteration": last["comm_bytes"] / max(last["num_linear_solves"], 1) / 1e6,
            "split": dict({k: last[k] for k in ("n_ranks", "n_owned_captures", "n_top_tiles", "split_top_work",
                                                "split_max_rank_work", "split_total_work")},
                          active_ranks=last["n_active_ranks"]),
            "transport": ("host all-reduce callback over gloo, ranks sharing cuda:" + str(device) +
                          " (test transport: no scaling measurement)") if callback else
                         ("RCCL, one GPU per rank" if world > 1 else
                          "RCCL, one-rank communicator, multi-rank path forced (debug)" if args.rccl_one_rank else None),
            "phase_ms_per_solve": {k: phased[f"t_{k}_ms"] for k in
                                   ("linearize", "schur", "cholesky", "solve", "backsub", "cost")},
            "roofline": roofline,
            "cpu_baseline": None,
            "library": lm.library_info(),
        }
        if not args.no_fingerprint:   # which kind of MI355X box this line ran on (a few ms, untimed)
            out["box_fingerprint"] = lm.box_fingerprint(device)
        if world == 1 and not args.no_incremental and args.config == "cfg3":
            print("bench: incremental cfg2 flow", file=sys.stderr, flush=True)
            out["incremental_cfg2"] = bench_incremental("cfg2")
            # the same flow eliminating every capture (rounds 3-5's default)
            out["incremental_cfg2_captures"] = bench_incremental("cfg2", elimination=1)
        if world == 1 and args.config == "cfg3" and not args.no_localize:
            print("bench: cfg5 localize batch", file=sys.stderr, flush=True)
            out["localize_cfg5"] = bench_localize(args, world, rank, side=True)
        if world == 1 and not args.no_cpu_baseline:
            # every CPU this process is granted: the box gives one GPU's share of the node
            # (OMP_NUM_THREADS, 16 on the GPU box) while nproc / lscpu report the whole node
            # (recorded beside it); more threads than the share only oversubscribe it
            host = host_cpu_info()
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or min(host["nproc"], 16)
            print(f"bench: CPU baseline on {threads} threads", file=sys.stderr, flush=True)
            out["cpu_baseline"] = cpu_baseline(g, threads, args.config)
            out["cpu_baseline"]["host_cpu"] = host
            out["cpu_baseline"]["cgroup_cpu_quota"] = host["cgroup_cpu_quota"]
            if args.config == "cfg3":   # plus the reference's own setting (Ceres num_threads = 1) on cfg2
                out["cpu_baseline_cfg2_1_thread"] = cpu_baseline(synth.config_graph("cfg2"), 1, "cfg2")
        print(json.dumps(out), flush=True)
    if world > 1 or args.rccl_one_rank:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
