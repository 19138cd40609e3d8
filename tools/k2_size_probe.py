"""K2 size probe (development aid): time to optimal of uniform random
instances (bench.py's k2_instance) at growing n, to pick the strong-scaling
workload; K1-wide beside it where its table fits.
    python tools/k2_size_probe.py n1 n2 ... [--seeds 1,2]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import k2_instance  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
seeds = [1]
for a in sys.argv[1:]:
    if a.startswith("--seeds="):
        seeds = [int(s) for s in a.split("=", 1)[1].split(",")]
ctx = tspgpu.Context(device=0)
for n in [int(a) for a in args]:
    for seed in seeds:
        d = k2_instance(n, seed)
        t = time.perf_counter()
        cost, tour, st = tspgpu.search_solve(ctx, d)
        wall = (time.perf_counter() - t) * 1e3
        line = (f"n={n} seed={seed} cost={cost:.6f} wall={wall:.2f} ms kernel={st['kernel_ms']:.3f} ms "
                f"nodes={st['nodes']:.3e} rounds={st['rounds']} |O|={st['optimal_tours']}")
        if n <= 26:
            w = ctx.solve_instance(d)
            line += f" | K1-wide {w[2]:.3f} ms agree={w[0] == cost}"
        print(line, flush=True)
