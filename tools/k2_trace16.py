"""The reference's `./tsp 16 1` instance solved REPS times through
tspgpu.search_solve (development aid: run under rocprofv3 --kernel-trace to
get the chain's per-kernel durations and the gaps between them)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
tspgpu.tune_from_environ()
from bench import Shard  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
ctx = tspgpu.Context(device=0)
d = Shard(16, 1, 0, 1).distances()[0]
for _ in range(reps):
    c, tour, st = tspgpu.search_solve(ctx, d)
print(c, st["kernel_ms"], st.get("bb_nodes", st.get("nodes")))
