"""K2 hard-instance scan (development aid): time to optimal over seeds of
uniform (bench.k2_instance) or clustered random instances, to pick a
strong-scaling workload.   python tools/k2_seed_scan.py n seeds [clusters]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import k2_instance  # noqa: E402

n, seeds = int(sys.argv[1]), int(sys.argv[2])
clusters = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ctx = tspgpu.Context(device=0)
rows = []
for seed in range(1, seeds + 1):
    if clusters:
        rng = np.random.default_rng(seed)
        cx = rng.uniform(100, 900, size=(clusters, 2))
        xy = cx[np.arange(n) % clusters] + rng.normal(0, 50, size=(n, 2))
        d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
    else:
        d = k2_instance(n, seed)
    t = time.perf_counter()
    cost, tour, st = tspgpu.search_solve(ctx, d)
    wall = (time.perf_counter() - t) * 1e3
    rows.append((wall, seed, st["kernel_ms"], st["nodes"]))
    print(f"n={n} clusters={clusters} seed={seed} wall={wall:.2f} ms kernel={st['kernel_ms']:.3f} ms "
          f"nodes={st['nodes']:.3e}", flush=True)
rows.sort(reverse=True)
print("hardest:", rows[:3])
