"""Build the HIP extension libarslam_lm.so in-tree (gfx950).

The product is a plain C-ABI shared library (include/arslam_lm.h) compiled
by hipcc; nothing is JIT-compiled at import time, so the .so built here
travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.environ.get("ARSLAM_LIB") or os.path.join(HERE, "libarslam_lm.so")   # (override: variant builds)
SOURCES = ["lm_kernels.hip", "dense_llt.hip", "lm_solver.hip", "debug_api.hip", "llt_plan.cpp",
           "host_structure.cpp", "localize.hip"]
HOST = os.path.join(HERE, "host")
HOST_SOURCES = ["yaml_lite.cpp", "ar_slam_solver.cpp", "slam_capi.cpp"]   # plain C++ (g++)
ARCH = os.environ.get("ARSLAM_ARCH", "gfx950")


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HOST, f) for f in os.listdir(HOST)] + \
        [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    """Compile libarslam_lm.so if any source is newer.  Safe under concurrent callers (torchrun
    ranks): one process builds behind an exclusive file lock while the others wait, and the
    library is written to a private path and renamed into place, so a reader never maps a
    half-written file."""
    if not force and not _stale():
        return LIB
    import fcntl
    with open(os.path.join(HERE, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and not _stale():   # another process built it while we waited
            return LIB
        return _build_locked(verbose)


def build_id():
    """What a built library is made of, embedded in it (arslam_lm_version): the git commit of the
    tree (+dirty when the sources differ from it; "nogit" outside a checkout) and a digest of every
    source, header and extra flag, so any measurement or fault can be attributed to its build."""
    import hashlib
    h = hashlib.sha256(os.environ.get("ARSLAM_EXTRA_FLAGS", "").encode())
    files = [os.path.join(CSRC, f) for f in SOURCES] + [os.path.join(HOST, f) for f in HOST_SOURCES] + \
        sorted(os.path.join(d, f) for d in (CSRC, HOST, os.path.join(ROOT, "include"))
               for f in os.listdir(d) if f.endswith((".h", ".hpp")))
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.relpath(f, ROOT).encode() + b"\0" + fh.read())
    commit = "nogit"
    try:
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True, timeout=10).stdout.strip() or "nogit"
        if commit != "nogit":
            rel = [os.path.relpath(f, ROOT) for f in files]
            dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--"] + rel, capture_output=True,
                                   text=True, timeout=10).stdout.strip()
            commit += "+dirty" if dirty else ""
    except (OSError, subprocess.SubprocessError):
        pass
    return f"{commit} src {h.hexdigest()[:12]}"


def _build_locked(verbose):
    extra = os.environ.get("ARSLAM_EXTRA_FLAGS", "")
    objdir = os.path.join(HERE, "_obj" + ("_" + "".join(c for c in extra if c.isalnum()) if extra else ""))
    os.makedirs(objdir, exist_ok=True)
    flags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
             "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
             f'-DARSLAM_BUILD_ID="{build_id()}"'] + os.environ.get("ARSLAM_EXTRA_FLAGS", "").split()
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc()] + flags + (["-x", "hip"] if src.endswith(".cpp") else []) + ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for src in HOST_SOURCES:
        obj = os.path.join(objdir, "host_" + os.path.splitext(src)[0] + ".o")
        cmd = ["g++", "-O2", "-fPIC", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
               "-I", HOST, "-c", os.path.join(HOST, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    errs = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            errs.append(f"--- {src} ---\n{out.decode()}")
        elif verbose and out:
            print(out.decode())
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    tmp = f"{LIB}.tmp{os.getpid()}"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", tmp] + objs + \
          ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
