"""A/B of library variants on one box (debug): each variant ar_slam_amd/var_<name>.so (or the
default library, name "base") runs in its own process, interleaved over rounds; per run it
prints the mean k_factor_dag launch (HIP events), LM iterations/s over timed cfg solves, the
final cost and a digest of the solved parameters (bit-identity across variants).
usage: python tools/ab.py cfg3 rounds name1 name2 ...   (a name env:VAR=VALUE: the default library under that switch)      (child: --child cfg lib steps)"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg, steps):
    sys.path.insert(0, ROOT)
    import numpy as np
    from ar_slam_amd import lm, synth
    g = synth.config_graph(cfg)
    lm.warm_up()
    rp = lm.ResidentProblem(camera=g.camera, cap=g.cap, tag=g.tag, obs_cap=g.obs_cap, obs_tag=g.obs_tag,
                            corners=g.corners, kernel_timing=1,
                            phase_timing=int(os.environ.get("AB_PHASES", "0")))   # (AB_PHASES=1: per-phase device ms)
    rp.solve()
    t0 = time.perf_counter()
    ss = [rp.solve() for _ in range(steps)]
    el = time.perf_counter() - t0
    it = sum(s["num_linear_solves"] for s in ss)
    dom = sum(s["t_dominant_ms"] for s in ss) / max(1, sum(s["n_dominant_launches"] for s in ss))
    h = hashlib.sha256(np.ascontiguousarray(rp.camera).tobytes() + np.ascontiguousarray(rp.cap).tobytes() +
                       np.ascontiguousarray(rp.tag).tobytes()).hexdigest()[:12]
    li = lm.library_info()
    ph = {k[2:-3]: round(sum(s[k] for s in ss) / len(ss), 4) for k in
          ("t_linearize_ms", "t_schur_ms", "t_cholesky_ms", "t_solve_ms", "t_backsub_ms")}
    print(json.dumps({"factor_us": dom * 1e3, "it_s": it / el, "cost": repr(ss[-1]["final_cost"]), "digest": h,
                      "lib": f"{li['file']} sha {li['sha256']}", "build": li["build"], "phases": ph}))


def main():
    cfg, rounds, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    res = {n: [] for n in names}
    for r in range(rounds):
        for n in names:
            env = dict(os.environ)
            if n.startswith("env:"):   # the default library under environment switches: env:NAME=VALUE[,NAME=VALUE]
                for kv in n[4:].split(","):
                    k, v = kv.split("=", 1)
                    env[k] = v
            elif n != "base":
                env["ARSLAM_LIB"] = os.path.join(ROOT, "ar_slam_amd", f"var_{n}.so")
            out = subprocess.run([sys.executable, __file__, "--child", cfg, "8"], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:   # (the library is named even when the child failed)
                lib = env.get("ARSLAM_LIB") or os.path.join(ROOT, "ar_slam_amd", "libarslam_lm.so")
                so = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:12] if os.path.exists(lib) else "missing"
                print(n, "FAILED", f"lib {os.path.basename(lib)} sha {so}", out.stdout[-1000:], out.stderr[-600:],
                      flush=True)
                continue
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[n].append(d)
            print(f"round {r} {n:12s} factor {d['factor_us']:7.1f} us  {d['it_s']:7.1f} it/s  cost {d['cost']}  {d['digest']}"
                  f"  [{d['lib']}, build {d['build']}]" + (f"  phases {d['phases']}" if os.environ.get("AB_PHASES") else ""),
                  flush=True)
    for n in names:
        if not res[n]:
            continue
        f = sorted(x["factor_us"] for x in res[n])
        i = sorted(x["it_s"] for x in res[n])
        print(f"{n:12s} factor median {f[len(f) // 2]:7.1f} us (min {f[0]:.1f})  it/s median {i[len(i) // 2]:7.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
    else:
        main()
