"""Debug: load the task graph written by ARSLAM_DAG_DUMP (debug_reduced_plan)."""
import numpy as np


def load(path):
    f = open(path, "rb")
    n, nw, T, ni, ntg = np.frombuffer(f.read(40), np.int64)
    d = {"n": int(n), "T": int(T)}
    d["tasks"] = np.frombuffer(f.read(16 * n), np.int32).reshape(n, 4)
    d["woff"] = np.frombuffer(f.read(4 * (n + 1)), np.int32)
    d["waits"] = np.frombuffer(f.read(8 * nw), np.int32).reshape(nw, 2)
    d["sub"] = np.frombuffer(f.read(8 * n), np.int32).reshape(n, 2)
    d["tmap"] = np.frombuffer(f.read(4 * T * T), np.int32).reshape(T, T)
    d["items"] = np.frombuffer(f.read(16 * ni), np.int32).reshape(ni, 4)
    d["targets"] = np.frombuffer(f.read(8 * ntg), np.int32).reshape(ntg, 2)
    d["cont"] = np.frombuffer(f.read(4 * n), np.int32)
    d["maxdep"] = np.frombuffer(f.read(4 * n), np.int32)
    d["nt"] = int(d["tmap"].max()) + 1
    return d
