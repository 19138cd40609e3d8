"""K1 variant-4 parent-store cache policy sweep (development aid).

Each library variant (lib/libtspgpu<suffix>.so, built with -DTSPGPU_PAR_AUX=a)
runs in its own child process (TSPGPU_LIB); costs and tours must match across
variants bit for bit.  Usage: python tools/k1_policy.py [suffixes...]"""
import hashlib, os, subprocess, sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, os.path.join(HERE, "tsp-mpi-reduction_amd"))
    import numpy as np
    import tspgpu

    ctx = tspgpu.Context(device=0)
    sizes = [(16, 16384)] if os.environ.get("K1P_N16") else [(16, 16384), (15, 16384), (14, 16384)]
    for n, B in sizes:
        rng = np.random.default_rng(n)
        xy = rng.uniform(0, 1000, size=(B, n, 2))
        d = np.sqrt(((xy[:, :, None, :] - xy[:, None, :, :]) ** 2).sum(-1))
        # the context's own buffers and stream, timed by the ABI's HIP events (as bench.py)
        dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
        for _ in range(2):
            ctx.solve_device(dd, n, B, dc, dt, ctx.stream)
        ctx.synchronize()
        reps = 20 if os.environ.get("K1P_N16") else 8
        ctx.timer_start()
        for _ in range(reps):
            ctx.solve_device(dd, n, B, dc, dt, ctx.stream)
        ms = ctx.timer_stop() / reps
        ctx.synchronize()
        h = hashlib.sha1(ctx.download(dc, (B,), np.float64).tobytes()
                         + ctx.download(dt, (B, n + 1), np.int32).tobytes()).hexdigest()[:12]
        tb = tspgpu.table_bytes_per_block(n) * B
        print(f"lib={os.path.basename(os.environ.get('TSPGPU_LIB', 'default'))} n={n} B={B} {ms:.3f} ms "
              f"{B / ms * 1e3:.3e} blocks/s {tb / ms / 1e9:.3f} TB/s(alg) hash={h} grid={ctx.last_grid()}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    pols = sys.argv[1:] or ["", "_aux2", "_aux16", "_head", ""]
    rc = 0
    for p in pols:
        env = dict(os.environ, TSPGPU_LIB=os.path.join(HERE, "tsp-mpi-reduction_amd", "lib", f"libtspgpu{p}.so"))
        r = subprocess.run([sys.executable, "-u", __file__, "child"], env=env, timeout=120)
        if r.returncode != 0:
            rc = r.returncode
            break
    sys.exit(rc)
