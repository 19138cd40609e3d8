"""test_tree_bound_keeps_the_answer[clustered]'s searches one by one, timed,
with the block-local chained levels on and off (development aid)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402

ctx = tspgpu.Context(device=0)
rng = np.random.default_rng(12)
for n in (18, 22, 25):
    c = rng.uniform(100, 900, size=(3, 2))
    xy = c[np.arange(n) % 3] + rng.normal(0, 40, size=(n, 2))
    d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
    for local in (0, 1):
        for mst, minrem in (("0", None), ("1", None), ("1", "0")):
            tspgpu.untune()
            tspgpu.tune("CHAIN_LOCAL", local)
            tspgpu.tune("SEARCH_MST", float(mst))
            if minrem is not None:
                tspgpu.tune("SEARCH_MST_MINREM", float(minrem))
            t = time.perf_counter()
            cost, tour, st = tspgpu.search_solve(ctx, d)
            print(f"n={n} local={local} mst={mst} minrem={minrem}: {time.perf_counter() - t:.3f} s cost {cost:.6f} "
                  f"nodes {st['nodes']} rounds {st['rounds']} kernel {st['kernel_ms']:.1f} ms", flush=True)
ctx.close()
