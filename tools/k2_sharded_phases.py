"""Host/device split of one sharded K2 solve (search_dist.solve_sharded, the
path bench.py's k2_strong_scaling measures) at N = 1, per host phase
(stats["host_phases_ms"]), next to its kernel time and the native
tspgpu_search_solve.  Prints one JSON line per instance.

    python tools/k2_sharded_phases.py [n seed] ...   (default: 32 35 and the 16-city golden)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402

tspgpu.tune_from_environ()
import bench  # noqa: E402
import search_dist  # noqa: E402

ctx = tspgpu.Context(device=0)
args = [int(x) for x in sys.argv[1:]] or [32, 35, 32, 14, 24, 5, 16, 0]
for n, seed in zip(args[0::2], args[1::2]):
    d = bench.Shard(16, 1, 0, 1).distances()[0] if n == 16 and seed == 0 else bench.k2_instance(n, seed)
    for bound in ("device", "host"):
        rows = []
        for _ in range(6):
            t = time.perf_counter()
            cost, tour, st = search_dist.solve_sharded(ctx, d, bound=bound)
            rows.append(((time.perf_counter() - t) * 1e3, st))
        rows.sort(key=lambda r: r[0])
        wall, st = rows[len(rows) // 2]
        # the native one-process search with the device bound extended to this size, and without
        tspgpu.tune("SEARCH_DEVICE_BOUND_MAXN", "33" if bound == "device" else "20")
        nat = []
        for _ in range(6):
            t = time.perf_counter()
            c2, t2, s2 = tspgpu.search_solve(ctx, d)
            nat.append(((time.perf_counter() - t) * 1e3, s2["kernel_ms"], s2["nodes"]))
        tspgpu.untune("SEARCH_DEVICE_BOUND_MAXN")
        nat.sort()
        print(json.dumps({"n": n, "seed": seed, "bound": bound, "cost": cost,
                          "sharded_wall_ms_median": round(wall, 3), "sharded_wall_ms_best": round(rows[0][0], 3),
                          "kernel_ms": round(st["kernel_ms"], 4), "nodes": st["nodes"],
                          "wall_over_kernel": round(wall / st["kernel_ms"], 3),
                          "host_phases_ms": {k: round(v, 3) for k, v in st["host_phases_ms"].items()},
                          "native_wall_ms_median": round(nat[len(nat) // 2][0], 3),
                          "native_kernel_ms": round(nat[len(nat) // 2][1], 4), "native_nodes": nat[len(nat) // 2][2],
                          "same": bool(c2 == cost and list(t2) == list(tour))}), flush=True)
