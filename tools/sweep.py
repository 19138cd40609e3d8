"""Kernel tuning sweep (development aid): K1 launch time per configuration.

    python tools/sweep.py [n ...]
Each configuration is a fresh context created under TSPGPU_THREADS /
TSPGPU_WG_PER_CU; all configurations run interleaved in one process.
SWEEP_I32=1 runs the integer-distance K1 on the rounded matrices.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402

ns = [int(a) for a in sys.argv[1:]] or [16, 14, 12]
# (K1 variant, threads, workgroups per CU); SWEEP="v,t,w;v,t,w" overrides
configs = [(0, 512, 2), (1, 256, 4), (1, 256, 8), (1, 512, 2), (1, 512, 4), (1, 1024, 2)]
if os.environ.get("SWEEP"):
    configs = [tuple(int(x) for x in c.split(",")) for c in os.environ["SWEEP"].split(";")]
for n in ns:
    B = {16: 8192, 15: 16384, 14: 16384, 13: 32768, 12: 65536}.get(n, 65536)
    shard = Shard(n, B, 0, B)
    d = shard.distances()
    i32 = os.environ.get("SWEEP_I32") == "1"
    vb = 4 if i32 else 8
    if i32:
        d = np.rint(d).astype(np.int32)
    rows = []
    ctxs = []
    for v, th, wg in configs:
        tspgpu.tune("K1", str(v))
        tspgpu.tune("THREADS", str(th))
        tspgpu.tune("WG_PER_CU", str(wg))
        ctx = tspgpu.Context(device=0)
        ctxs.append((v, th, wg, ctx, ctx.upload(d), ctx.alloc(B * vb), ctx.alloc(B * (n + 1) * 4)))
    ref = None
    for rep in range(2):
        for v, th, wg, ctx, dd, dc, dt in ctxs:
            solve = ctx.solve_device_i32 if i32 else ctx.solve_device
            solve(dd, n, B, dc, dt, ctx.stream)
            ctx.timer_start()
            for _ in range(3):
                solve(dd, n, B, dc, dt, ctx.stream)
            ms = ctx.timer_stop() / 3
            c = ctx.download(dc, (B,), np.int32 if i32 else np.float64)
            if ref is None:
                ref = c
            ok = np.array_equal(c, ref)
            if rep == 1:
                relax = tspgpu.relaxations_per_block(n) * B
                tb = tspgpu.table_bytes_per_block(n) * B * vb / 8
                print(f"n={n} B={B} {'i32' if i32 else 'f64'} k1={v} threads={th} wg/cu={wg} grid={ctx.last_grid()} {ms:.3f} ms "
                      f"{B / ms * 1e3:.3e} blocks/s {relax / ms / 1e9:.3f} Trelax/s {tb / ms / 1e6:.0f} GB/s alg "
                      f"{'ok' if ok else 'MISMATCH'}", flush=True)
    for *_, ctx, dd, dc, dt in ctxs:
        for p in (dd, dc, dt):
            ctx.free(p)
        ctx.close()
