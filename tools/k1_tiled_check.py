"""K1 variant 5 (sub-cube tiled) on the GPU: parity against the CPU oracle for
every configuration in hkt_cfg.h, then device time per launch next to the
variant-4 kernel (development aid; the parity tests proper are in tests/).

    python tools/k1_tiled_check.py [blocks] [cfg ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

CFGS = {0: (16, 8), 1: (16, 8), 2: (16, 8), 3: (16, 8), 4: (16, 8), 5: (15, 8), 6: (15, 8), 7: (16, 4), 8: (16, 4),
        9: (15, 4), 10: (14, 8), 11: (16, 8), 12: (16, 8), 13: (16, 8), 14: (16, 8), 15: (16, 8), 16: (16, 8), 17: (16, 8), 18: (16, 8), 19: (16, 4),
        20: (16, 4), 21: (16, 4), 22: (15, 8), 23: (14, 8), 24: (15, 4), 25: (13, 8), 26: (13, 8),
        27: (15, 4), 28: (14, 4)}
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
which = [int(x) for x in sys.argv[2:]] or sorted(CFGS)


def ctx_for(variant, cfg=None):
    os.environ["TSPGPU_K1"] = str(variant)
    if cfg is None:
        os.environ.pop("TSPGPU_TILED_CFG", None)
    else:
        os.environ["TSPGPU_TILED_CFG"] = str(cfg)
    return tspgpu.Context(device=0)


def parity_blocks(n, count, seed):
    rng = np.random.default_rng(seed)
    blocks = []
    for b in range(count):
        if b % 3 == 0:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)  # heavy ties
        elif b % 3 == 1:
            xy = rng.integers(0, 40, size=(n, 2)).astype(np.float64)
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        blocks.append([(b * n + i, xy[i, 0], xy[i, 1]) for i in range(n)])
    return tspgpu.distance_matrix(blocks)


def timed(ctx, d, n, vb, reps=5):
    Bn = d.shape[0]
    dd = ctx.upload(d)
    dc, dt = ctx.alloc(Bn * 8), ctx.alloc(Bn * (n + 1) * 4)
    fn = ctx.solve_device if vb == 8 else ctx.solve_device_i32
    fn(dd, n, Bn, dc, dt, ctx.stream)
    ctx.synchronize()
    ctx.timer_start()
    for _ in range(reps):
        fn(dd, n, Bn, dc, dt, ctx.stream)
    ms = ctx.timer_stop() / reps
    cost = ctx.download(dc, (Bn,), np.float64 if vb == 8 else np.int32)
    tour = ctx.download(dt, (Bn, n + 1), np.int32)
    for p in (dd, dc, dt):
        ctx.free(p)
    return ms, cost, tour


results = {}
for n in sorted({CFGS[c][0] for c in which}):
    shard = Shard(n, B, 0, B)
    d = shard.distances()
    for vb in sorted({CFGS[c][1] for c in which if CFGS[c][0] == n}):
        dv = d if vb == 8 else np.rint(d).astype(np.int32)
        ref_ctx = ctx_for(4 if (n == 16 and vb == 8) else 2)
        ms_ref, c_ref, t_ref = timed(ref_ctx, dv, n, vb)
        ref_ctx.close()
        relax = tspgpu.relaxations_per_block(n) * B
        print(f"n={n} vb={vb} B={B} baseline variant: {ms_ref:.3f} ms/launch {relax / ms_ref / 1e9:.3f} Trelax/s",
              flush=True)
        for cfg in which:
            if CFGS[cfg] != (n, vb):
                continue
            ctx = ctx_for(5, cfg)
            # parity vs the oracle on tie-heavy + random blocks
            pd = parity_blocks(n, 96, 1234 + cfg)
            if vb == 4:
                pd = np.rint(pd).astype(np.int32)
                pc, pt = ctx.solve_blocks_i32(pd)
            else:
                pc, pt = ctx.solve_blocks(pd)
            bad = 0
            for b in range(pd.shape[0]):
                oc, ot = O.solve_block(np.asarray(pd[b], dtype=np.float64))
                if float(pc[b]) != oc or pt[b][:n + 1].tolist() != ot:
                    bad += 1
                    if bad <= 3:
                        print(f"  cfg {cfg} MISMATCH block {b}: gpu {pc[b]!r} {pt[b].tolist()} oracle {oc!r} {ot}")
            ms, c5, t5 = timed(ctx, dv, n, vb)
            same = bool(np.array_equal(c5, c_ref) and np.array_equal(t5, t_ref))
            print(f"  cfg {cfg}: parity {96 - bad}/96, full batch equal to baseline: {same}, "
                  f"{ms:.3f} ms/launch {relax / ms / 1e9:.3f} Trelax/s ({ms_ref / ms:.2f}x) grid={ctx.last_grid()}",
                  flush=True)
            ctx.close()
