"""K2 static-shard balance on ONE GPU (development aid): every shard r of W
run alone with the same start bound as the sharded search (no exchange), so
max over r of the shard's time predicts the W-GPU time to optimal and
sum / max its parallel efficiency.
    python tools/k2_shard_balance.py n seed [W ...] [--depth=D,...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import k2_instance  # noqa: E402

n, seed = int(sys.argv[1]), int(sys.argv[2])
Ws = [int(w) for w in sys.argv[3:] if not w.startswith("--")] or [1, 2, 4, 8]
depths = [0]
for a_ in sys.argv[3:]:
    if a_.startswith("--depth="):
        depths = [int(x) for x in a_.split("=", 1)[1].split(",")]
d = k2_instance(n, seed)
ctx = tspgpu.Context(device=0)
ub, _ = tspgpu.heuristic_tour(d)
for depth, W in [(dp, w) for dp in depths for w in Ws]:
    walls, kms, nodes = [], [], []
    for r in range(W):
        S = tspgpu.Search(ctx, d, shard=r, nshards=W, depth=depth)
        try:
            S.set_bound(ub)
            t = time.perf_counter()
            S.start()
            steps = 0
            while S.step():
                steps += 1
            walls.append((time.perf_counter() - t) * 1e3)
            kms.append(S.timing()[0])
            nodes.append(S.counters()[1])
            used_depth = S.depth
        finally:
            S.close()
    print(f"n={n} seed={seed} depth={used_depth} W={W}: shard wall ms max {max(walls):.2f} sum {sum(walls):.2f} "
          f"(eff {sum(walls) / (W * max(walls)):.2f}); kernel ms max {max(kms):.2f} sum {sum(kms):.2f}; "
          f"nodes {sum(nodes):.3e} max/mean {max(nodes) * W / max(sum(nodes), 1):.2f}", flush=True)
