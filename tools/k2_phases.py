"""Where K2's in-process time to optimal goes (development aid): the
reference's `./tsp 16 1` instance (and a 32-city one) solved through the
public ABI step by step, every phase timed on the host:
heuristic bound, search creation (host tables, Lagrangian/tree weights,
device buffers), start (seeds + suffix table), each frontier step (launch +
count readback), records and the tie rule.  Prints one JSON line per instance.

    python tools/k2_phases.py [reps]
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


def phases(ctx, d):
    t = {}
    t0 = time.perf_counter()
    ub, _ = tspgpu.heuristic_tour(d)
    t1 = time.perf_counter()
    S = tspgpu.Search(ctx, d)
    t2 = time.perf_counter()
    S.set_bound(ub)
    S.start()
    t3 = time.perf_counter()
    steps = []
    while True:
        a = time.perf_counter()
        more = S.step()
        steps.append((time.perf_counter() - a) * 1e3)
        if not more:
            break
    t4 = time.perf_counter()
    inc, nodes, recs = S.counters()
    rec = S.records(inc)
    cost = tspgpu.bits_cost(inc, S.dtype)
    tour = tspgpu.select_tour(d, rec, cost)
    t5 = time.perf_counter()
    kms, rounds = S.timing()
    S.close()
    t6 = time.perf_counter()
    t.update(heuristic_ms=(t1 - t0) * 1e3, create_ms=(t2 - t1) * 1e3, start_ms=(t3 - t2) * 1e3,
             steps_ms=(t4 - t3) * 1e3, step_ms=steps, records_select_ms=(t5 - t4) * 1e3,
             destroy_ms=(t6 - t5) * 1e3, total_ms=(t6 - t0) * 1e3, kernel_ms=kms, rounds=rounds,
             nodes=nodes, cost=cost, tour=[int(x) for x in tour])
    return t


VARIANTS = [{}, {"TSPGPU_SEARCH_CHAIN": "0"}, {"TSPGPU_SEARCH_LAGRANGE": "0"}]


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--variants":
        import subprocess
        for v in VARIANTS:
            out = subprocess.run([sys.executable, __file__, "5"], env=dict(os.environ, **v), capture_output=True,
                                 text=True, timeout=120).stdout
            for ln in out.splitlines():
                if ln.startswith("{"):
                    d = json.loads(ln)
                    d.pop("tour", None)
                    d.pop("step_ms", None)
                    print(json.dumps(dict(env=v, **d)), flush=True)
        return
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ctx = tspgpu.Context(device=0)
    cases = {"tsp16_1": Shard(16, 1, 0, 1).distances()[0], "rand32_s35": np.asarray(k2_instance(32, 35))}
    for name, d in cases.items():
        runs = [phases(ctx, d) for _ in range(reps)]
        best = min(runs, key=lambda r: r["total_ms"])
        c, tr, st = tspgpu.search_solve(ctx, d)
        walls = []
        for _ in range(reps):
            t = time.perf_counter()
            tspgpu.search_solve(ctx, d)
            walls.append((time.perf_counter() - t) * 1e3)
        best["search_solve_ms"] = min(walls)
        best["search_solve_median_ms"] = sorted(walls)[len(walls) // 2]
        best["search_solve_stats"] = {k: st[k] for k in ("nodes", "rounds", "kernel_ms", "phases", "fallback")
                                      if k in st}
        best["same_as_search_solve"] = bool(c == best["cost"] and list(tr) == best["tour"])
        print(json.dumps(dict(instance=name, **best)), flush=True)


if __name__ == "__main__":
    main()
