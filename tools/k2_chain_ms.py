"""Kernel time of the 16-city chain alone (development aid for timing-only
builds whose answers are wrong): Search + set_bound + chain, S.timing()."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

ctx = tspgpu.Context(device=0)
d = Shard(16, 1, 0, 1).distances()[0]
ub, _ = tspgpu.heuristic_tour(d)
ks = []
for _ in range(20):
    S = tspgpu.Search(ctx, d)
    S.set_bound(ub)
    S.chain()
    ks.append(S.timing()[0])
    S.close()
ks.sort()
print(json.dumps({"kernel_ms_best": ks[0], "kernel_ms_median": ks[len(ks) // 2]}))
