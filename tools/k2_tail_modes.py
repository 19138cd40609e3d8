"""K2 B&B register-tail modes (development aid): TSPGPU_SEARCH_TAIL = 0 (DFS to
the leaves), 5 or 6 (prefixes with 5/6 cities left folded by tail_kernel).
Same instances as tools/k2_time.py; answers checked against K1 / K1-wide."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402  (reference generator)

ctx = tspgpu.Context(device=0)
ns = [int(a) for a in sys.argv[1:]] or [14, 16, 18, 20]
for n in ns:
    sh = Shard(n, 4, 0, 4)
    d = sh.distances()
    ref = ctx.solve_blocks(d) if n <= 16 else None
    for b in range(4):
        want = (ref[0][b], ref[1][b][:n + 1].tolist()) if ref else ctx.solve_instance(d[b])[:2]
        for mode in ("0", "5", "6"):
            tspgpu.tune("SEARCH_TAIL", mode)
            best = None
            for rep in range(3):
                t = time.perf_counter()
                cost, tour, st = tspgpu.search_solve(ctx, d[b])
                wall = (time.perf_counter() - t) * 1e3
                if best is None or st["kernel_ms"] < best[1]["kernel_ms"]:
                    best = (wall, st, cost, list(tour))
            wall, st, cost, tour = best
            ok = cost == want[0] and tour == list(want[1])
            print(f"n={n} b={b} tail={mode} ok={ok} wall={wall:.2f} ms kernel={st['kernel_ms']:.3f} ms "
                  f"nodes={st['nodes']:.3e} {st['nodes'] / max(st['kernel_ms'], 1e-9) / 1e9:.3f} Tnodes/s "
                  f"rounds={st['rounds']} |O|={st['optimal_tours']}", flush=True)
