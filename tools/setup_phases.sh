#!/bin/bash
# cfg3 cold setup, phase by phase (ARSLAM_SETUP_PROFILE), three loads in one process
set -o pipefail
mkdir -p gpurun_out
ARSLAM_SETUP_PROFILE=1 timeout -k 10 200 python - > gpurun_out/setup_phases.txt 2>&1 <<'PY' || { tail -20 gpurun_out/setup_phases.txt; exit 1; }
import sys, time
sys.path.insert(0, ".")
from ar_slam_amd import lm, synth
g = synth.config_graph("cfg3")
lm.device_count()
for i in range(3):
    t = time.perf_counter()
    rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners, device=0)
    print(f"load {i}: {1e3 * (time.perf_counter() - t):.1f} ms", file=sys.stderr, flush=True)
    del rp
PY
cat gpurun_out/setup_phases.txt
