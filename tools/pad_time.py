"""Time the n=16 default K1 launch (16384 blocks) with the per-block slot
padded by each given byte count (TSPGPU_SLOT_PAD; layout experiment).
    python tools/pad_time.py PAD ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard  # noqa: E402

B = 16384
d = Shard(16, B, 0, B).distances()
ctx = tspgpu.Context(device=0)
dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * 17 * 4)
for pad in sys.argv[1:]:
    tspgpu.tune("SLOT_PAD", pad)
    ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
    ctx.timer_start()
    for _ in range(5):
        ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
    print(f"pad={pad} variant={ctx.last_variant()} {ctx.timer_stop() / 5:.3f} ms/launch", flush=True)
