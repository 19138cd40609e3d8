"""Quick device-time probe of the K1 kernel at several n (development aid)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tsp-mpi-reduction_amd"))
import numpy as np
import torch
import tspgpu

ctx = tspgpu.Context(device=0, slots=int(os.environ.get("SLOTS", "0")))
for n, B in [(12, 8192), (14, 2048), (16, 2048), (16, 1)]:
    rng = np.random.default_rng(0)
    xy = rng.uniform(0, 1000, size=(B, n, 2))
    # fast distance matrix for timing only (numpy); parity runs use libm via the ABI
    d = np.sqrt(((xy[:, :, None, :] - xy[:, None, :, :]) ** 2).sum(-1))
    dd = torch.from_numpy(d).cuda(); dc = torch.empty(B, dtype=torch.float64, device="cuda")
    dt = torch.empty((B, n + 1), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(2):
        ctx.solve_device(dd.data_ptr(), n, B, dc.data_ptr(), dt.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for _ in range(reps):
        ctx.solve_device(dd.data_ptr(), n, B, dc.data_ptr(), dt.data_ptr(), s.cuda_stream)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    relax = tspgpu.relaxations_per_block(n) * B
    tb = tspgpu.table_bytes_per_block(n) * B
    print(f"n={n} B={B} grid={ctx.last_grid()} {ms:.3f} ms/launch  {B/ms*1e3:.3e} blocks/s  {relax/ms/1e9:.3f} Trelax/s  {tb/ms/1e9:.3f} TB/s(alg)", flush=True)
