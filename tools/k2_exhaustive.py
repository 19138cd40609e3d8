"""Config-2 probe (development aid): `./tsp n 1 1000 1000` by exhaustive
enumeration (K2 with the bound off), time and nodes/s."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tsp-mpi-reduction_amd"), ROOT]
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

ctx = tspgpu.Context(device=0)
for n in [int(a) for a in sys.argv[1:]] or [12, 13, 14]:
    d = Shard(n, 1, 0, 1).distances()[0]
    for rep in range(2):
        t = time.perf_counter()
        cost, tour, st = tspgpu.search_solve(ctx, d, exhaustive=True)
        wall = (time.perf_counter() - t) * 1e3
    c2, t2, _ = tspgpu.search_solve(ctx, d)
    print(f"n={n} cost={cost!r} wall={wall:.1f} ms kernel={st['kernel_ms']:.1f} ms nodes={st['nodes']:.3e} "
          f"{st['nodes'] / (st['kernel_ms'] * 1e-3) / 1e9:.1f} G nodes/s rounds={st['rounds']} "
          f"lane_util={st['active_steps'] / max(st['lane_steps'], 1):.3f} same_as_bnb={c2 == cost and list(t2) == list(tour)}",
          flush=True)
