"""K2 tree-bound probe (development aid): time to optimal with the Held-Karp
tree bound on and off (TSPGPU_SEARCH_MST, read when a search is created),
same cost and tour required, and K1-wide's answer where it fits (n <= 25).
    python tools/k2_tree_probe.py n:seed[:off] ...   (":off" also runs MST=0)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import k2_instance  # noqa: E402

ctx = tspgpu.Context(device=0)


def run(d, mst):
    tspgpu.tune("SEARCH_MST", "1" if mst else "0")
    tspgpu.search_solve(ctx, d) if d.shape[0] <= 20 else None  # warm (small cases only)
    t = time.perf_counter()
    cost, tour, st = tspgpu.search_solve(ctx, d)
    return cost, list(map(int, tour)), (time.perf_counter() - t) * 1e3, st


for arg in sys.argv[1:]:
    parts = arg.split(":")
    n, seed = int(parts[0]), int(parts[1])
    d = k2_instance(n, seed)
    modes = [True, False] if len(parts) > 2 else [True]
    res = {m: run(d, m) for m in modes}
    c1, t1, w1, s1 = res[True]
    line = f"n={n} seed={seed} cost={c1:.6f} MST: wall={w1:.2f} ms kernel={s1['kernel_ms']:.3f} ms nodes={s1['nodes']:.3e} rounds={s1['rounds']}"
    if False in res:
        c0, t0, w0, s0 = res[False]
        line += f" | no MST: wall={w0:.2f} ms kernel={s0['kernel_ms']:.3f} ms nodes={s0['nodes']:.3e} agree={c0 == c1 and t0 == t1}"
    if n <= 25:
        cw, tw, _ = ctx.solve_instance(np.asarray(d, dtype=np.float64))
        line += f" | K1-wide agree={cw == c1 and list(map(int, tw)) == t1}"
    print(line, flush=True)
