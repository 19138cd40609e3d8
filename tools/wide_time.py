"""K1-wide timing probe (development aid): single instances over the whole GPU."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tsp-mpi-reduction_amd"), ROOT]
import numpy as np
import tspgpu
from bench import Shard  # noqa: E402

ctx = tspgpu.Context(device=0)
for n in [int(a) for a in sys.argv[1:]] or [12, 16, 20, 24]:
    rng = np.random.default_rng(n)
    xy = rng.uniform(0, 1000, size=(n, 2))
    d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
    best = None
    for _ in range(3):
        t = time.perf_counter()
        cost, tour, ms = ctx.solve_instance(d)
        wall = (time.perf_counter() - t) * 1e3
        best = min(best or 1e30, ms)
    line = f"n={n} cost={cost:.6f} wide kernel={best:.3f} ms wall={wall:.3f} ms"
    if n <= 20:
        dd = ctx.upload(d[None]); dc = ctx.alloc(8); dt = ctx.alloc((n + 1) * 4)
        ctx.solve_device(dd, n, 1, dc, dt, ctx.stream); ctx.synchronize()
        ctx.timer_start()
        for _ in range(5):
            ctx.solve_device(dd, n, 1, dc, dt, ctx.stream)
        k1 = ctx.timer_stop() / 5
        line += f"  K1 one-workgroup kernel={k1:.3f} ms"
    print(line, flush=True)
