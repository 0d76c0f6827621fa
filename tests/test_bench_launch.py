"""bench.py's multi-GPU launcher on the CPU box: `python bench.py --gpus 2` with no torchrun
environment starts its two rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE, a 127.0.0.1
rendezvous), and `--launch-check` makes the ranks meet over gloo without touching a GPU, so the
launch path the driver's N-GPU runs take is exercised here.  (The solve itself through the same
launcher runs in tests/test_gpu_multirank.py::test_bench_launches_its_ranks.)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                         timeout=180, env=e, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_gpus_flag_starts_the_ranks():
    d = _run("--gpus", "2", "--launch-check")
    assert d["launch_check"] and d["n_gpus"] == 2 and d["ranks"] == [0, 1]
    assert d["env"]["MASTER_ADDR"] == "127.0.0.1"


def test_gpus_flag_four_ranks():
    d = _run("--gpus", "4", "--launch-check")
    assert d["n_gpus"] == 4 and d["ranks"] == [0, 1, 2, 3]


def test_one_gpu_starts_no_children():
    d = _run("--gpus", "1", "--launch-check")
    assert d["n_gpus"] == 1 and d["ranks"] == [0] and d["env"]["LOCAL_WORLD_SIZE"] is None


def test_a_dead_rank_ends_the_launch():
    """A rank that exits before the rendezvous must not leave rank 0 waiting in it forever: the
    launcher polls every rank, ends the others at the first non-zero exit and returns that status."""
    import time
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e["ARSLAM_LAUNCH_CHECK_FAIL_RANK"] = "1"
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-check"],
                         capture_output=True, text=True, timeout=120, env=e, cwd=ROOT)
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert time.time() - t0 < 60
