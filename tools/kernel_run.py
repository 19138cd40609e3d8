"""Run the K1 kernel a few times on one shard (profiling target, no torch).

    python tools/kernel_run.py [n] [blocks] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
shard = Shard(n, B, 0, B)
d = shard.distances()
ctx = tspgpu.Context(device=0)
dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
ctx.timer_start()
for _ in range(reps):
    ctx.solve_device(dd, n, B, dc, dt, ctx.stream)
print(f"n={n} B={B} reps={reps} {ctx.timer_stop() / reps:.3f} ms/launch grid={ctx.last_grid()}")
