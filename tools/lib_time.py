"""Device time of K1 n=16 (16384 blocks) for library builds x tiled configs.
    python tools/lib_time.py LIBNAME[,LIBNAME...] CFG[,CFG...]
LIBNAME is a file in tsp-mpi-reduction_amd/lib (each run in a fresh process)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--one":
    sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
    sys.path.insert(0, ROOT)
    import tspgpu
    from bench import Shard
    B = 16384
    d = Shard(16, B, 0, B).distances()
    for cfg in sys.argv[3].split(","):
        tspgpu.tune("K1", "5")
        tspgpu.tune("TILED_CFG", cfg)
        ctx = tspgpu.Context(device=0)
        dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * 17 * 4)
        ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
        ctx.timer_start()
        for _ in range(5):
            ctx.solve_device(dd, 16, B, dc, dt, ctx.stream)
        ms = ctx.timer_stop() / 5
        print(f"lib={sys.argv[2]} cfg={cfg} variant={ctx.last_variant()} {ms:.3f} ms/launch", flush=True)
        for p in (dd, dc, dt):
            ctx.free(p)
        ctx.close()
    sys.exit(0)
for lib in sys.argv[1].split(","):
    path = os.path.join(ROOT, "tsp-mpi-reduction_amd", "lib", lib)
    subprocess.run([sys.executable, __file__, "--one", lib, sys.argv[2]], env=dict(os.environ, TSPGPU_LIB=path),
                   check=True, timeout=200)
