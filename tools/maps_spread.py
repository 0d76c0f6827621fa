"""Debug: the device's distance from the oracle driver on the map-file and cfg1 flows, beside the
distance between the oracle's two exact arithmetics (Schur vs full normal equations), per solve:
cost (relative), focal (px), centres (m, after rigid alignment), RMS (relative).  Input for the
tolerance caps of tests/test_gpu_maps.py.  usage: python tools/maps_spread.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import yaml  # noqa: E402

from ar_slam_amd import lm, synth  # noqa: E402
from oracle.driver import OracleSlam  # noqa: E402
import test_gpu_maps as T  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def dev(s, o, alt):
    last = s.last_summary()
    ref, oth = T._state(o), T._state(alt)
    q = T._points(ref[2], ref[3])
    p_ours = T._align_rigid(T._points(s.capture_poses(), s.aruco_poses()), q)
    p_alt = T._align_rigid(T._points(oth[2], oth[3]), q)
    rms = lambda c, n: np.sqrt(2 * c / (4 * n))   # noqa: E731
    return {"cost_rel": [abs(last["final_cost"] - ref[0]) / ref[0], abs(oth[0] - ref[0]) / ref[0]],
            "focal_px": [abs(s.camera()[0][0] - ref[1]), abs(oth[1] - ref[1])],
            "centres_m": [float(np.max(np.abs(p_ours - q))), float(np.max(np.abs(p_alt - q)))],
            "termination": [last["termination"], o.last_summary["termination"]]}


out = {}
for name in ["cfg1", "tiny", "small"]:
    if name == "cfg1":
        doc = yaml.safe_load(open(os.path.join(GOLDEN, "cfg1_map.yaml")))
    else:
        doc = T._write_map(synth.config_graph(name), f"/tmp/map_{name}.yaml")
    path = os.path.join(GOLDEN, "cfg1_map.yaml") if name == "cfg1" else f"/tmp/map_{name}.yaml"
    s = lm.SlamSolver()
    s.load_yaml(path)
    s.solve()
    o = OracleSlam(camera=doc["camera"]["params"])
    alt = OracleSlam(camera=doc["camera"]["params"], elimination=1)
    for x in (o, alt):
        for uid, ids, corners in T._messages(doc):
            x.add_detections(uid, ids, corners)
        x.solve()
    out[f"map_{name}"] = dev(s, o, alt)
doc = yaml.safe_load(open(os.path.join(GOLDEN, "cfg1_map.yaml")))
s = lm.SlamSolver()
o = OracleSlam(camera=doc["camera"]["params"])
alt = OracleSlam(camera=doc["camera"]["params"], elimination=1)
s.set_camera(doc["camera"]["params"])
for i, (uid, ids, corners) in enumerate(T._messages(doc)):
    s.add_detections(uid, ids, corners)
    s.solve_incremental()
    for x in (o, alt):
        x.add_detections(uid, ids, corners)
        x.solve_incremental()
    out[f"cfg1_incremental_msg{i}"] = dev(s, o, alt)
print(json.dumps(out, indent=1))
