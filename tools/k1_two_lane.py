"""K1 at the bench size (./tsp 16 65536 1000 1000) as one launch pair on one
context, against the same blocks split over 2 or 4 contexts whose launch
pairs run concurrently on their own streams (development aid, round 6: two
ranks sharing one GPU ran a step in 23.9 ms where one rank takes 25.3).
Prints one JSON line per mode: wall per step (median of REPS) and whether
every cost equals the one-launch run's."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

n, B = 16, 65536
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
d = Shard(n, B, 0, B).distances()
ctxs = [tspgpu.Context(device=0) for _ in range(4)]
dd = ctxs[0].upload(d)
dc, dt = ctxs[0].alloc(B * 8), ctxs[0].alloc(B * (n + 1) * 4)
ref = None
for lanes in (4, 2, 1, 2, 4, 1):
    per = B // lanes
    ts = []
    for r in range(reps + 1):
        t = time.perf_counter()
        for k in range(lanes):
            c = ctxs[k]
            c.solve_device(dd + k * per * n * n * 8, n, per, dc + k * per * 8, dt + k * per * (n + 1) * 4, c.stream)
        for k in range(lanes):
            ctxs[k].synchronize()
        if r:
            ts.append((time.perf_counter() - t) * 1e3)
    cost = ctxs[0].download(dc, (B,), np.float64)
    if ref is None and lanes == 1:
        ref = cost.copy()
    ts.sort()
    print(json.dumps({"lanes": lanes, "blocks_per_lane": per, "ms_per_step_median": round(ts[len(ts) // 2], 3),
                      "ms_best": round(ts[0], 3), "same_costs_as_one_launch": None if ref is None else bool((cost == ref).all())}),
          flush=True)
