"""K2 sharded-driver probe (development aid): the device tie key path at
several sizes, one process (world 1), with the driver's statistics, and the
time to the optimal tour of the reference's 16-city instance through
search_dist.solve_sharded against tspgpu_search_solve."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tsp-mpi-reduction_amd")]
import numpy as np  # noqa: E402

import search_dist  # noqa: E402
import tspgpu  # noqa: E402
from bench import Shard, k2_instance  # noqa: E402

ctx = tspgpu.Context(device=0)
for n, seed in ((22, 7), (26, 7), (22, 3), (24, 1)):
    d = np.asarray(k2_instance(n, seed))
    c0, t0, s0 = tspgpu.search_solve(ctx, d)
    S = tspgpu.Search(ctx, d)
    ub, _ = tspgpu.heuristic_tour(d)
    S.set_bound(ub)
    ok = S.chain()
    inc, nodes, recs = S.counters()
    slot = S.tie_slot(inc)
    rc, tt = tspgpu.tie_tour(d, slot[1], slot[2], tspgpu.bits_cost(inc, tspgpu.F64)) if slot[0] else (None, None)
    key = tspgpu.tie_key(t0)
    S.close()
    c, t, st = search_dist.solve_sharded(ctx, d)
    print(f"n={n} seed={seed}: solve tie={s0['tie']} checked={s0['tie_checked']} | chain={ok} slot={slot} "
          f"key(t0)={key} tie_tour rc={rc} same={tt is not None and list(tt) == list(t0)} | sharded tie={st['tie']} "
          f"gather={st['record_gather']} same={c == c0 and list(t) == list(t0)}", flush=True)
d16 = Shard(16, 1, 0, 1).distances()[0]
for name, fn in (("search_solve", lambda: tspgpu.search_solve(ctx, d16)),
                 ("solve_sharded", lambda: search_dist.solve_sharded(ctx, d16))):
    best = 1e9
    for _ in range(20):
        t = time.perf_counter()
        c, tour, st = fn()
        best = min(best, (time.perf_counter() - t) * 1e3)
    print(f"16-city {name}: best of 20 {best:.3f} ms, tie={st.get('tie')} gather={st.get('record_gather')}", flush=True)
ctx.close()
