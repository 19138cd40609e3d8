"""Config-2 probe: `./tsp n 1 1000 1000` by exhaustive enumeration —
enum.hip (default) vs the round kernels with the bound off
(TSPGPU_ENUM_KERNEL=0); kernel time, nodes/s, same answer."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tsp-mpi-reduction_amd"), ROOT]
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402

ctx = tspgpu.Context(device=0)
old = os.environ.get("OLD", "1") == "1"
for n in [int(a) for a in sys.argv[1:]] or [12, 13, 14, 15]:
    d = Shard(n, 1, 0, 1).distances()[0]
    res = {}
    for mode in (("enum", "old") if old and n <= 15 else ("enum",)):
        tspgpu.tune("ENUM_KERNEL", "1" if mode == "enum" else "0")
        best = None
        for rep in range(3):
            t = time.perf_counter()
            cost, tour, st = tspgpu.search_solve(ctx, d, exhaustive=True)
            wall = (time.perf_counter() - t) * 1e3
            if best is None or st["kernel_ms"] < best[2]["kernel_ms"]:
                best = (cost, tour, st, wall)
        cost, tour, st, wall = best
        res[mode] = (cost, list(tour))
        print(f"n={n} {mode:4s} cost={cost!r} wall={wall:.2f} ms kernel={st['kernel_ms']:.3f} ms "
              f"nodes={st['nodes']:.4e} {st['nodes'] / (st['kernel_ms'] * 1e-3) / 1e12:.2f} T nodes/s "
              f"tours={st['records']} recs depth={st['depth']}", flush=True)
    if len(res) == 2:
        print(f"n={n} same answer: {res['enum'] == res['old']}", flush=True)
