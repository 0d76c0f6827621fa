"""Print the LM traces of one config under several reduced orderings (GPU)."""
import sys
sys.path.insert(0, ".")
from ar_slam_amd import lm, synth

name = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
g = synth.config_graph(name)
for skip, ordering in [(1, 0), (1, 1), (1, 2), (0, 2)]:
    cam, cap, tag, s = lm.solve_graph(g, cholesky_skip_zero_tiles=skip, reduced_ordering=ordering)
    print(f"skip={skip} ordering={ordering} term={s['termination']}/{s['rule']} "
          f"iters={len(s['iterations'])} solves={s['num_linear_solves']} final={s['final_cost']:.12e} f={cam[0]:.9f}")
    for it in s["iterations"]:
        print(f"   {it['iteration']:3d} cost={it['cost']:.15e} dcost={it['cost_change']:.3e} rho={it['relative_decrease']:.6f}"
              f" radius={it['trust_region_radius']:.3e} step={it['step_norm']:.3e} |g|={it['gradient_max_norm']:.3e}"
              f" ok={it['step_is_successful']}")
