"""Chained vs stepwise K2 search above 18 cities (development aid):
search_solve wall and device time on uniform instances of 19..32 cities
(bench.k2_instance seeds) with TSPGPU_CHAIN_MAXN=18 (stepwise) and 32
(chained, overflow falls back to stepwise), one subprocess per setting."""
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
from bench import k2_instance
ctx = tspgpu.Context(device=0)
out = {{}}
for n, seed in ((20, 1), (24, 2), (28, 3), (32, 35), (32, 14), (32, 30)):
    d = np.asarray(k2_instance(n, seed))
    tspgpu.search_solve(ctx, d)
    walls = []
    for _ in range(5):
        t = time.perf_counter()
        c, tour, st = tspgpu.search_solve(ctx, d)
        walls.append((time.perf_counter() - t) * 1e3)
    out["%d_%d" % (n, seed)] = dict(best=round(min(walls), 3), dev=round(st["kernel_ms"], 3), rounds=st["rounds"],
                                    nodes=st["nodes"], cost=c, tour=hash(tuple(tour.tolist())))
print(json.dumps(out))
'''


def main():
    for maxn in (18, 32):
        env = dict(os.environ, TSPGPU_CHAIN_MAXN=str(maxn))
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                           timeout=120)
        res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-400:]
        print(json.dumps(dict(maxn=maxn, rc=r.returncode, res=res)), flush=True)


if __name__ == "__main__":
    main()
