"""The reference's real flow on a BASELINE config: ArSlamSolver::solveIncremental
(ar_slam_util.cpp:629-742), i.e. one full ceres::Solve of the whole problem so
far after every capture (:736), through the C++ host mirror and the pointer-keyed
C-ABI.  Reports the wall time of the whole flow, the number of Solve calls, and
per call the setup (host structure, ordering, tile plan, upload: summary
setup_time_s) and the minimizer time.  usage: bench_incremental.py [cfg2]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ar_slam_amd import build, lm, synth  # noqa: E402

build.build()
name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
g = synth.config_graph(name)
# the process's HIP runtime started outside the timed flow, as in bench.py (whose cfg3 solves run
# first): a throwaway solver over the first two captures
w = lm.SlamSolver()
w.set_camera(g.camera)
for c in range(2):
    sel = g.obs_cap == c
    w.add_detections(f"cap{c}", [f"tag_{t}" for t in g.obs_tag[sel]], g.corners[sel])
    w.solve_incremental()
del w
# (default options, as a drop-in user gets them; ARSLAM_PHASES=1: per-phase device times)
# (ARSLAM_ELIM: the elimination option, e.g. 3 = Ceres' exact mixed set)
s = lm.SlamSolver(phase_timing=int(os.environ.get("ARSLAM_PHASES", "0")),
                  elimination=int(os.environ.get("ARSLAM_ELIM", "0")))
s.set_camera(g.camera)
t0 = time.perf_counter()
t_add = 0.0
for c in range(g.n_cap):
    sel = g.obs_cap == c
    ta = time.perf_counter()
    s.add_detections(f"cap{c}", [f"tag_{t}" for t in g.obs_tag[sel]], g.corners[sel])
    t_add += time.perf_counter() - ta
    s.solve_incremental()
wall = time.perf_counter() - t0
n = s.num_solves
setup = mini = 0.0
iters = 0
kinds = [0, 0, 0]
phase = [0.0] * 5   # summary.setup_phase_s summed over the full loads
PH = ("t_linearize_ms", "t_schur_ms", "t_cholesky_ms", "t_solve_ms", "t_backsub_ms", "t_cost_ms")
ph = dict.fromkeys(PH, 0.0)
for i in range(n):
    d = s.solve_summary(i)
    for k in PH:
        ph[k] += d.get(k, 0.0)
    kinds[d["setup_kind"]] += 1
    if d["setup_kind"] == 0:
        phase = [a + b for a, b in zip(phase, d.get("setup_phase_s", [0.0] * 5))]
    setup += d["setup_time_s"]
    mini += d["minimizer_time_s"]
    iters += d["num_linear_solves"]
last = s.last_summary()
if os.environ.get("ARSLAM_INC_DUMP"):   # debug: one line per Solve
    with open(os.environ["ARSLAM_INC_DUMP"], "w") as f:
        for i in range(n):
            d = s.solve_summary(i)
            f.write(json.dumps({k: d[k] for k in ("elimination_used", "setup_kind", "setup_time_s", "minimizer_time_s",
                                                  "num_linear_solves", "n_factor_tiles", "n_levels", "n_reduced",
                                                  "order_reused", "t_cholesky_ms")}) + "\n")
print(json.dumps({"flow": f"solveIncremental, {name}: {g.n_cap} captures / {g.n_tag} tags, one message per capture",
                  "wall_s": wall, "solves": n, "lm_iterations": iters,
                  "setup_ms_per_solve": 1e3 * setup / n, "minimizer_ms_per_solve": 1e3 * mini / n,
                  "other_ms_per_solve": 1e3 * (wall - setup - mini) / n,
                  "add_detections_ms_per_message": 1e3 * t_add / g.n_cap,
                  "device_phase_ms_per_solve": {k[2:-3]: round(v / n, 4) for k, v in ph.items()},
                  "setup_kinds": {"load": kinds[0], "values": kinds[1], "append": kinds[2]},
                  "elimination_used": {str(k): int(v) for k, v in zip(*np.unique(
                      [s.solve_summary(i)["elimination_used"] for i in range(n)], return_counts=True))},
                  "load_setup_phase_ms": {k: round(1e3 * v / max(1, kinds[0]), 4) for k, v in
                                          zip(("structure", "order", "plan", "upload", "rest"), phase)},
                  "final_rms_px": last["final_rms_px"], "final_termination": last["termination"],
                  "last_plan": {k: last[k] for k in ("n_factor_tiles", "n_levels", "n_update_tiles",
                                                     "factor_scalar_flops", "n_reduced")}}))
