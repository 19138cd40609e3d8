"""The reference's 16-city instance (./tsp 16 1 1000 1000) through
tspgpu.search_solve under knob settings (development aid): kernel time
(device clock, median of REPS), nodes, the answer against the default.

    python tools/k2_16_sweep.py [REPS]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tsp-mpi-reduction_amd"))
sys.path.insert(0, ROOT)
import tspgpu  # noqa: E402
from bench import Shard  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
ctx = tspgpu.Context(device=0)
d = Shard(16, 1, 0, 1).distances()[0]
c0, t0, _ = tspgpu.search_solve(ctx, d)
SETS = json.loads(os.environ["SETS_JSON"]) if os.environ.get("SETS_JSON") else [{}] if os.environ.get("DEFAULT_ONLY") else [{}, {"SEARCH_DEPTH": 5}, {"SEARCH_DEPTH": 6}, {"SEARCH_DEPTH": 3}, {"SEARCH_TAIL": 5},
        {"SEARCH_DEPTH": 5, "SEARCH_TAIL": 5}, {"CHAIN_LOCAL": 1, "CHAIN_LOCAL_FPB": 32},
        {"CHAIN_GRID": 1}, {"CHAIN_GRID": 4}, {"CHAIN_FPB": 128}]
for knobs in SETS:
    for k, v in knobs.items():
        tspgpu.tune(k, str(v))
    try:
        ks, ws, nodes, same = [], [], 0, True
        for _ in range(reps):
            t_0 = time.perf_counter()
            c, t, st = tspgpu.search_solve(ctx, d)
            ws.append((time.perf_counter() - t_0) * 1e3)
            ks.append(st["kernel_ms"])
            nodes = st["nodes"]
            same = same and c == c0 and list(t) == list(t0)
        ks.sort()
        print(json.dumps({"knobs": knobs, "lib": os.path.basename(tspgpu.LIB_PATH) if hasattr(tspgpu, "LIB_PATH") else None,
                          "cost": c0, "kernel_ms_median": round(ks[len(ks) // 2], 4),
                          "kernel_ms_best": round(ks[0], 4), "in_process_ms_median": round(sorted(ws)[len(ws) // 2], 4), "nodes": nodes, "depth": st.get("depth"),
                          "same_answer": same}), flush=True)
    except tspgpu.TspGpuError as e:
        print(json.dumps({"knobs": knobs, "error": str(e)}), flush=True)
    finally:
        for k in knobs:
            tspgpu.untune(k)
