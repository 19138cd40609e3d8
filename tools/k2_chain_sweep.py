"""Chained K2 search geometry sweep (development aid): the reference's
`./tsp 16 1` instance and two more 16-18 city ones, solved in process under
TSPGPU_CHAIN_FPB (paths per block run) x TSPGPU_CHAIN_GRID (blocks per CU),
one subprocess per setting; best-of-reps wall and device span per setting.

    python tools/k2_chain_sweep.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, json, numpy as np
sys.path.insert(0, "{root}/tsp-mpi-reduction_amd"); sys.path.insert(0, "{root}")
import tspgpu
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
from bench import Shard
ctx = tspgpu.Context(device=0)
cases = {{"tsp16_1": Shard(16, 1, 0, 1).distances()[0]}}
rng = np.random.default_rng(3)
for n in (17, 18):
    xy = rng.uniform(0, 1000, size=(n, 2))
    cases["u%d" % n] = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
out = {{}}
for name, d in cases.items():
    tspgpu.search_solve(ctx, d)
    walls, dev = [], []
    for _ in range(15):
        t = time.perf_counter()
        c, tour, st = tspgpu.search_solve(ctx, d)
        walls.append((time.perf_counter() - t) * 1e3)
        dev.append(st["kernel_ms"])
    out[name] = dict(best=round(min(walls), 4), med=round(sorted(walls)[7], 4), dev=round(min(dev), 4), cost=c,
                     tour=hash(tuple(tour.tolist())))
print(json.dumps(out))
'''


def main():
    settings = [(int(a), int(b)) for a, b in (x.split(":") for x in sys.argv[1:])] or \
        [(f, g) for f in (1024, 512, 256) for g in (1, 2, 3, 4)]
    for fpb, grid in settings:
        env = dict(os.environ, TSPGPU_CHAIN_FPB=str(fpb), TSPGPU_CHAIN_GRID=str(grid))
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True,
                           text=True, timeout=60)
        res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-300:]
        print(json.dumps(dict(fpb=fpb, grid=grid, rc=r.returncode, res=res)), flush=True)


if __name__ == "__main__":
    main()
