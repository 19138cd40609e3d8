"""Run one K1 large-batch launch configuration a few times (target for
rocprofv3 --pmc passes; development aid):  python tools/k1_once.py n B vb variant[:cfg]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402

n, B, vb = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
v, _, cfg = sys.argv[4].partition(":")
tspgpu.tune("K1", v)
if cfg:
    tspgpu.tune("TILED_CFG", cfg)
d = Shard(n, B, 0, B).distances()
if vb == 4:
    d = np.rint(d).astype(np.int32)
ctx = tspgpu.Context(device=0)
dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
fn = ctx.solve_device if vb == 8 else ctx.solve_device_i32
for _ in range(int(os.environ.get("REPS", "2"))):
    fn(dd, n, B, dc, dt, ctx.stream)
ctx.synchronize()
print("variant", ctx.last_variant())
