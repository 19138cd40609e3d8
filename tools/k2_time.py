"""K2 timing probe (development aid): one-shot search of single instances."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import tspgpu
from bench import Shard  # noqa: E402  (reference generator)

ctx = tspgpu.Context(device=0)
ns = [int(a) for a in sys.argv[1:]] or [12, 14, 16, 18]
for n in ns:
    sh = Shard(n, 4, 0, 4)
    d = sh.distances()
    for b in range(4):
        t = time.perf_counter()
        cost, tour, st = tspgpu.search_solve(ctx, d[b])
        wall = (time.perf_counter() - t) * 1e3
        print(f"n={n} b={b} cost={cost:.6f} wall={wall:.2f} ms kernel={st['kernel_ms']:.3f} ms nodes={st['nodes']:.3e} "
              f"{st['nodes'] / max(st['kernel_ms'], 1e-9) / 1e6:.3f} Gnodes/s depth={st['depth']} items={st['items']} "
              f"|O|={st['optimal_tours']} recs={st['records']} phases={st['phases']} rounds={st['rounds']}", flush=True)
    c1, t1 = ctx.solve_blocks(d) if n <= 20 else (None, None)
    if c1 is not None:
        print(f"   K1 agrees: {all(tspgpu.search_solve(ctx, d[b])[0] == c1[b] for b in range(4))}", flush=True)
