"""One search: the clustered 25-city instance of test_tree_bound_keeps_the_answer
with the tree bound off (development aid; TSPGPU_LIB picks the library)."""
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
    if n != int(sys.argv[1] if len(sys.argv) > 1 else 25):
        continue
    tspgpu.tune("SEARCH_MST", 0.0)
    t = time.perf_counter()
    cost, tour, st = tspgpu.search_solve(ctx, d)
    print(f"{os.environ.get('TSPGPU_LIB', 'tree')}: n={n} mst=0: {time.perf_counter() - t:.3f} s cost {cost:.6f} "
          f"nodes {st['nodes']} rounds {st['rounds']} phases {st.get('phases')} kernel {st['kernel_ms']:.1f} ms",
          flush=True)
ctx.close()
