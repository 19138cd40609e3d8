"""What the first K1 solve of each size pays for its kernels' code object
(verdict r05 item 8: is splitting the library per kernel family worth it?).

Each case runs in a FRESH process: context create, the transfer path warmed
with a 4-city solve (loads the small-n kernels' code object), then the first
and second one-block solve of size n; "first - second" is what the first use
of that size's code object (plus its host tables) costs.  Prints one JSON
line per case, with the size of the code object the case loads.

    python tools/startup_split_probe.py            (driver: spawns the cases)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)


def case(n):
    import numpy as np

    import tspgpu
    from bench import Shard

    t0 = time.perf_counter()
    ctx = tspgpu.Context(device=0)
    t1 = time.perf_counter()
    d4 = Shard(4, 1, 0, 1).distances()
    ctx.solve_blocks(np.ascontiguousarray(d4))
    t2 = time.perf_counter()
    d = np.ascontiguousarray(Shard(n, 1, 0, 1).distances())
    ts = []
    for _ in range(3):
        a = time.perf_counter()
        ctx.solve_blocks(d)
        ts.append((time.perf_counter() - a) * 1e3)
    return {"n": n, "ctx_create_ms": (t1 - t0) * 1e3, "warm_4city_first_ms": (t2 - t1) * 1e3,
            "first_ms": ts[0], "second_ms": ts[1], "third_ms": ts[2], "first_minus_third_ms": ts[0] - ts[2]}


if __name__ == "__main__":
    if len(sys.argv) > 1:
        print(json.dumps(case(int(sys.argv[1]))), flush=True)
        sys.exit(0)
    for n in (12, 14, 15, 16, 16, 12, 14, 15, 16):
        p = subprocess.run([sys.executable, __file__, str(n)], capture_output=True, text=True, timeout=120)
        print(p.stdout.strip() or json.dumps({"n": n, "error": p.stderr[-400:]}), flush=True)
