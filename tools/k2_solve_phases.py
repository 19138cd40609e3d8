"""Host phases of tspgpu_search_solve on the reference's `./tsp 16 1` instance
(development aid): the library's SEARCH_DEBUG knob prints one line per solve
on stderr (create+bound, run, device, read, select+destroy); this also times
the heuristic bound and the whole call from Python.

    python tools/k2_solve_phases.py [reps] 2> phases.log
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)

import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    d = Shard(n, 1, 0, 1).distances()[0]
    ctx = tspgpu.Context(device=0)
    for _ in range(3):
        tspgpu.search_solve(ctx, d)
    hs = []
    for _ in range(reps):
        t = time.perf_counter()
        tspgpu.heuristic_tour(d)
        hs.append((time.perf_counter() - t) * 1e3)
    hs.sort()
    print(f"n={n} heuristic_tour min {hs[0]:.3f} med {hs[len(hs) // 2]:.3f} ms")
    for knob in (None, 0):
        if knob is None:
            tspgpu.untune("SEARCH_DEVICE_BOUND")
        else:
            tspgpu.tune("SEARCH_DEVICE_BOUND", knob)
        ws = []
        tspgpu.tune("SEARCH_DEBUG", 1)
        for _ in range(reps):
            t = time.perf_counter()
            cost, tour, st = tspgpu.search_solve(ctx, d)
            ws.append((time.perf_counter() - t) * 1e3)
        tspgpu.untune("SEARCH_DEBUG")
        sys.stderr.flush()
        ws.sort()
        print(f"  device_bound={'default' if knob is None else knob}: search_solve min {ws[0]:.3f} "
              f"med {ws[len(ws) // 2]:.3f} ms; kernel {st['kernel_ms']:.3f} ms; nodes {st['nodes']}; "
              f"cost {cost!r}; tour {list(map(int, tour))}")
    ctx.close()


if __name__ == "__main__":
    main()
