"""Time the n=16 default K1 config of each ablation library (tools/abl_build.sh).
    python tools/abl_time.py MASK ...   (each mask runs in a fresh process)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
    sys.path.insert(0, ROOT)
    import numpy as np
    import tspgpu
    from bench import Shard
    B = 16384
    d = Shard(16, B, 0, B).distances()
    ctx = tspgpu.Context(device=0)
    dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * 17 * 4)
    ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
    ctx.timer_start()
    for _ in range(5):
        ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
    ms = ctx.timer_stop() / 5
    print(f"abl={sys.argv[2]} variant={ctx.last_variant()} {ms:.3f} ms/launch", flush=True)
    sys.exit(0)
for m in sys.argv[1:]:
    lib = os.path.join(ROOT, "tsp-mpi-reduction_amd", "lib", f"libtspgpu_abl{m}.so")
    subprocess.run([sys.executable, __file__, "--one", m], env=dict(os.environ, TSPGPU_LIB=lib), check=True, timeout=120)
