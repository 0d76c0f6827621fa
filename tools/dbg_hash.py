"""Debug: solve cfg3 twice with ARSLAM_FACTOR_HASH set and report the first
factorization / tiles whose bits differ (a data race in the executor)."""
import os
import sys
import numpy as np
sys.path.insert(0, '.')
path = "gpurun_out/hash.bin"
os.makedirs("gpurun_out", exist_ok=True)
if os.path.exists(path):
    os.remove(path)
os.environ["ARSLAM_FACTOR_HASH"] = path
from ar_slam_amd import lm, synth
g = synth.config_graph(sys.argv[1] if len(sys.argv) > 1 else "cfg3")
rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
runs = []
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    runs.append(rp.solve())
    print("solve", len(runs), runs[-1]["num_linear_solves"], runs[-1]["termination"], flush=True)
raw = np.fromfile(path, np.uint64)
recs, o = [], 0
while o < raw.size:
    nt, T = int(raw[o]), int(raw[o + 1])
    tmap = raw[o + 2:o + 2 + T * T].astype(np.int64).reshape(T, T)
    o += T * T
    recs.append((raw[o + 2:o + 2 + nt], raw[o + 2 + nt:o + 2 + nt + T]))
    o += 2 + nt + T
ik = {}
for i in range(T):
    for k in range(T):
        if tmap[i, k] >= 0:
            ik[int(tmap[i, k])] = (i, k)
nf = [r["num_linear_solves"] for r in runs]
print("linear solves per run", nf)
starts = np.cumsum([0] + nf)
for r in range(1, len(runs)):
    for f in range(min(nf[0], nf[r])):
        a, b = recs[starts[0] + f], recs[starts[r] + f]
        ds, dl = np.nonzero(a[0] != b[0])[0], np.nonzero(a[1] != b[1])[0]
        if len(ds) or len(dl):
            tiles = sorted(ik[int(t)] for t in ds)
            print(f"run {r} factorization {f}: {len(ds)} S tiles differ, "
                  f"{len(dl)} diagonal factors differ (cols {dl[:12]})")
            print("  differing tiles by column:", sorted(tiles, key=lambda x: (x[1], x[0]))[:24])
            break
    else:
        print(f"run {r}: identical factors")
