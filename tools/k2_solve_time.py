"""K2 search_solve wall time in process (development aid): the reference's
`./tsp 16 1` instance and a 32-city one, TSPGPU_SEARCH_DEBUG phase lines on
stderr, best/median wall over reps on stdout.

    TSPGPU_SEARCH_DEBUG=1 python tools/k2_solve_time.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard, k2_instance  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    ctx = tspgpu.Context(device=0)
    cases = {"tsp16_1": Shard(16, 1, 0, 1).distances()[0], "rand32_s35": np.asarray(k2_instance(32, 35))}
    for name, d in cases.items():
        tspgpu.search_solve(ctx, d)
        walls = []
        for _ in range(reps):
            t = time.perf_counter()
            c, tour, st = tspgpu.search_solve(ctx, d)
            walls.append((time.perf_counter() - t) * 1e3)
        print(json.dumps({"instance": name, "best_ms": min(walls), "median_ms": sorted(walls)[len(walls) // 2],
                          "kernel_ms": st["kernel_ms"], "tie": st["tie"], "tie_checked": st["tie_checked"],
                          "cost": c}), flush=True)


if __name__ == "__main__":
    main()
