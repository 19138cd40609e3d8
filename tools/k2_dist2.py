"""Two ranks on one GPU (gloo): where the sharded 16-city search's time goes
(development aid).  python -m torch.distributed.run --nproc-per-node 2
--master-addr 127.0.0.1 --master-port 29512 tools/k2_dist2.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tsp-mpi-reduction_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import search_dist  # noqa: E402
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
ctx = tspgpu.Context(device=0)
d = Shard(16, 1, 0, 1).distances()[0]
t = torch.zeros(7, dtype=torch.int64)
parts = [torch.empty_like(t) for _ in range(world)]
res = {}
for name, fn in (("all_gather_7", lambda: dist.all_gather(parts, t)),
                 ("search_create_chain", None), ("solve_sharded", lambda: search_dist.solve_sharded(ctx, d))):
    best = 1e9
    for _ in range(20):
        dist.barrier()
        t0 = time.perf_counter()
        if fn is None:
            S = tspgpu.Search(ctx, d, shard=rank, nshards=world)
            S.set_bound(tspgpu.heuristic_tour(d)[0])
            S.chain()
            S.close()
        else:
            fn()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    res[name] = round(best, 4)
print(rank, res, flush=True)
ctx.close()
dist.destroy_process_group()
