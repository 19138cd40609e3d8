"""Chained K2 levels: one launch per level against block-local levels
(expand_local_kernel) at several input runs per block (development aid).

    python tools/k2_local_sweep.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
from bench import Shard, k2_instance  # noqa: E402


def timed(ctx, d, reps):
    tspgpu.search_solve(ctx, d)
    ws, ks = [], []
    for _ in range(reps):
        t = time.perf_counter()
        c, tour, st = tspgpu.search_solve(ctx, d)
        ws.append((time.perf_counter() - t) * 1e3)
        ks.append(st["kernel_ms"])
    ws.sort()
    ks.sort()
    return c, ws[len(ws) // 2], ks[len(ks) // 2], st["nodes"], [int(x) for x in tour]


def main():
    ctx = tspgpu.Context(device=0)
    cases = [("tsp16_1", Shard(16, 1, 0, 1).distances()[0]), ("tsp14_1", Shard(14, 1, 0, 1).distances()[0])]
    for n, seed in ((20, 3), (24, 5), (32, 35)):
        cases.append((f"rand{n}_s{seed}", k2_instance(n, seed)))
    configs = [("per-level", {"CHAIN_LOCAL": 0})] + [(f"local fpb={f}", {"CHAIN_LOCAL_FPB": f}) for f in (8, 16, 32, 64)]
    for name, d in cases:
        ref = None
        for cname, knobs in configs:
            for k, v in knobs.items():
                tspgpu.tune(k, v)
            c, wall, kms, nodes, tour = timed(ctx, d, 9 if d.shape[0] <= 20 else 5)
            tspgpu.untune()
            if ref is None:
                ref = (c, tour)
            same = (c, tour) == ref
            print(f"{name:12s} {cname:14s} in-process {wall:7.3f} ms  kernels {kms:7.3f} ms  nodes {nodes:9d}  same {same}",
                  flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
