"""Dump one k_factor_dag task timeline of a cfg3 solve (debug; ARSLAM_DAG_TRACE must be set
before the library loads).  usage: ARSLAM_DAG_TRACE=out.bin python tools/trace_cfg3.py [cfg]"""
import sys

sys.path.insert(0, ".")
from ar_slam_amd import lm, synth  # noqa: E402

g = synth.config_graph(sys.argv[1] if len(sys.argv) > 1 else "cfg3")

cam, cap, tag, s = lm.solve_graph(g)
print("final cost", s["final_cost"], "iterations", len(s["iterations"]))
