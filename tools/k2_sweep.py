"""K2 sweep (development aid): one instance, several (kernel, refill, budget)
settings, each a fresh search.  K2SWEEP="k,refill,budget;..." (env)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
seeds = [int(s) for s in sys.argv[2:]] or [1]
cfgs = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("K2SWEEP", "2,8,256;1,8,256").split(";")]
ctx = tspgpu.Context(device=0)
for seed in seeds:
    xy = np.random.default_rng(seed).uniform(0, 1000, size=(n, 2))
    d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
    for kern, refill, budget in cfgs:
        tspgpu.tune("SEARCH_KERNEL", str(kern))
        tspgpu.tune("SEARCH_REFILL", str(refill))
        tspgpu.tune("SEARCH_BUDGET", str(budget))
        t = time.perf_counter()
        cost, tour, st = tspgpu.search_solve(ctx, d)
        wall = (time.perf_counter() - t) * 1e3
        print(f"n={n} seed={seed} kernel={kern} refill={refill} budget={budget} cost={cost:.6f} wall={wall:.1f} ms "
              f"kernel={st['kernel_ms']:.1f} ms nodes={st['nodes']:.3e} "
              f"{st['nodes'] / max(st['kernel_ms'], 1e-9) / 1e6:.2f} Gnodes/s rounds={st['rounds']} "
              f"lane_util={st['active_steps'] / max(st['lane_steps'], 1):.3f} steps={st['lane_steps'] / 64:.3e} "
              f"loads={st['item_loads']:.3e} nodes/active={st['nodes'] / max(st['active_steps'], 1):.2f}", flush=True)
