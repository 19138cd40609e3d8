"""K1 diagnostic build (TSPGPU_SUB_STAMP, tools/ab_build.sh): per-wave shader
clocks of the middle-pass bodies, their barriers, the edge intervals and the
whole block, read back from the tour words; prints medians over blocks and
waves.   TSPGPU_LIB=lib_ab/stamp.so python tools/k1_stamp.py [n] [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
tspgpu.tune("K1", 6)
d = Shard(n, B, 0, B).distances()
ctx = tspgpu.Context(device=0)
dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
for _ in range(3):
    ctx.solve_device(dd, n, B, dc, dt, ctx.stream)
ctx.synchronize()
raw = ctx.download(dt, (B, n + 1), np.int32)
t = raw[:, :16].astype(np.uint32).astype(np.float64).reshape(B, 4, 4)
rt = raw[:, 16].astype(np.uint32).astype(np.float64)
body, bar, edge, tot = (t[:, :, k] for k in range(4))
out = {"lib": os.path.basename(os.environ.get("TSPGPU_LIB", "libtspgpu.so")), "B": B,
       "median_cycles_per_block_wave": {"body": float(np.median(body)), "barrier": float(np.median(bar)),
                                        "edge": float(np.median(edge)), "total": float(np.median(tot))},
       "frac_of_total": {"body": float(np.median(body / tot)), "barrier": float(np.median(bar / tot)),
                         "edge": float(np.median(edge / tot))},
       "in_kernel_clock_ghz": float(np.median(tot[:, 0] / rt) * 0.1),
       "per_wave_body_median": [float(np.median(body[:, w])) for w in range(4)],
       "per_wave_barrier_median": [float(np.median(bar[:, w])) for w in range(4)]}
print(json.dumps(out))
