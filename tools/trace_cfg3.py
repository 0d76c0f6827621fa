"""Debug: dump one persistent-executor factorization timeline of a cfg3 solve
(ARSLAM_DAG_TRACE) and print its critical path and POTRF sub-phases."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
out = os.path.join(ROOT, "gpurun_out", "dag_trace.bin")
os.makedirs(os.path.dirname(out), exist_ok=True)
if os.path.exists(out):
    os.remove(out)
os.environ["ARSLAM_DAG_TRACE"] = out
os.environ.setdefault("ARSLAM_DAG_TRACE_SKIP", "2")
from ar_slam_amd import lm, synth  # noqa: E402
g = synth.config_graph(sys.argv[1] if len(sys.argv) > 1 else "cfg3")
rp = lm.ResidentProblem(g.camera, g.cap, g.tag, g.obs_cap, g.obs_tag, g.corners)
s = rp.solve()
print("solve", s["termination"], s["num_linear_solves"], "iterations")
for tool in ("dag_critical.py", "dag_phases.py", "dag_trace.py"):
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), out], check=True)
