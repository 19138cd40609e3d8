"""K2 on the reference's 16-city instance (./tsp 16 1 1000 1000, block 0):
search statistics under the current environment (TSPGPU_SEARCH_* knobs).
    python tools/k2_probe.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402

n = int(os.environ.get("K2_N", "16"))
d = Shard(n, 1, 0, 1).distances()[0]
ctx = tspgpu.Context(device=0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
if len(sys.argv) > 2:  # seed depth (the library reads TSPGPU_SEARCH_DEPTH when a search starts)
    tspgpu.tune("SEARCH_DEPTH", sys.argv[2])
for _ in range(reps):
    t = time.perf_counter()
    cost, tour, st = tspgpu.search_solve(ctx, d)
    wall = (time.perf_counter() - t) * 1e3
    st["wall_ms"] = round(wall, 3)
    st["cost"] = cost
    st["env"] = {k: v for k, v in os.environ.items() if k.startswith("TSPGPU_SEARCH")}
    print(json.dumps(st), flush=True)
print("heuristic", tspgpu.heuristic_tour(d)[0])
wide = ctx.solve_instance(d)
print("k1_wide", wide[0], "ms", wide[2])
