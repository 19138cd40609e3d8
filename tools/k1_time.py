"""K1 large-batch kernels on the GPU (development aid; the parity tests proper
are in tests/): for each requested (variant, configuration) the batch of
`./tsp n B 1000 1000` blocks is solved, compared bit for bit with variant 5's
default (costs and tours), and timed with HIP events on the context's stream
— the whole launch, then the forward and backtracking kernels apart.

    python tools/k1_time.py n B vb spec [spec ...]     spec = variant[:cfg], e.g. 6 5 6:65
Prints one JSON line per spec.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402


def ctx_for(variant, cfg=None):
    tspgpu.tune("K1", str(variant))
    if cfg is None:
        tspgpu.untune("TILED_CFG")
    else:
        tspgpu.tune("TILED_CFG", str(cfg))
    return tspgpu.Context(device=0)


def run(ctx, d, n, vb, reps):
    B = d.shape[0]
    dd = ctx.upload(d)
    dc, dt = ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
    fn = ctx.solve_device if vb == 8 else ctx.solve_device_i32
    fn(dd, n, B, dc, dt, ctx.stream)
    ctx.synchronize()
    ctx.timer_start()
    for _ in range(reps):
        fn(dd, n, B, dc, dt, ctx.stream)
    ms = ctx.timer_stop() / reps
    variant = ctx.last_variant()
    split = None
    if variant in (5, 6):
        ctx.k1_split_timing(True)
        fw, bt = [], []
        for _ in range(3):
            fn(dd, n, B, dc, dt, ctx.stream)
            f, b = ctx.k1_last_split_ms()
            fw.append(f)
            bt.append(b)
        ctx.k1_split_timing(False)
        split = (float(np.median(fw)), float(np.median(bt)))
    cost = ctx.download(dc, (B,), np.float64 if vb == 8 else np.int32)
    tour = ctx.download(dt, (B, n + 1), np.int32)
    for p in (dd, dc, dt):
        ctx.free(p)
    return ms, split, variant, cost, tour


def main():
    n, B, vb = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    specs = sys.argv[4:] or ["6", "5"]
    reps = int(os.environ.get("REPS", "5"))
    d = Shard(n, B, 0, B).distances()
    if vb == 4:
        d = np.rint(d).astype(np.int32)
    ref = ctx_for(5)
    _, _, _, c_ref, t_ref = run(ref, d, n, vb, 1)
    ref.close()
    relax = tspgpu.relaxations_per_block(n) * B
    for spec in specs:
        v, _, cfg = spec.partition(":")
        ctx = ctx_for(int(v), int(cfg) if cfg else None)
        ms, split, used, cost, tour = run(ctx, d, n, vb, reps)
        ctx.close()
        same = bool(np.array_equal(cost, c_ref) and np.array_equal(tour, t_ref))
        out = {"n": n, "B": B, "vb": vb, "spec": spec, "variant": used, "ms": ms, "trelax_s": relax / ms / 1e9,
               "same_as_v5": same}
        if split:
            out.update(forward_ms=split[0], backtrack_ms=split[1], forward_trelax_s=relax / split[0] / 1e9)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
