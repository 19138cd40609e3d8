"""Per-instance K2 solve timing of the tree-bound test's clustered cases, one
subprocess per (instance, env) with a time limit (development aid)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, json, numpy as np
sys.path.insert(0, "{root}/tsp-mpi-reduction_amd")
import tspgpu
tspgpu.tune_from_environ()  # (TSPGPU_<KNOB> variables of this tool -> library knobs)
n, seed_skip = {n}, {skip}
rng = np.random.default_rng(12)
for m in (18, 22, 25):
    c = rng.uniform(100, 900, size=(3, 2))
    xy = c[np.arange(m) % 3] + rng.normal(0, 40, size=(m, 2))
    if m == n:
        break
d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
ctx = tspgpu.Context(device=0)
t = time.perf_counter()
cost, tour, st = tspgpu.search_solve(ctx, d)
print(json.dumps(dict(n=n, ms=(time.perf_counter() - t) * 1e3, cost=cost, nodes=st["nodes"], records=st["records"],
                      tie=st["tie"], rounds=st["rounds"], kernel_ms=st["kernel_ms"])), flush=True)
'''


def main():
    for n in (18, 22, 25):
        for env in ({"TSPGPU_SEARCH_MST": "0"}, {"TSPGPU_SEARCH_MST": "0", "TSPGPU_SEARCH_TIE": "0"}):
            code = CHILD.format(root=ROOT, n=n, skip=0)
            t = time.perf_counter()
            try:
                r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, TSPGPU_SEARCH_DEBUG="2", **env),
                                   capture_output=True, text=True, timeout=40)
                out = r.stdout.strip().splitlines()[-1:] or [r.stderr[-400:]]
                steps = [ln for ln in r.stderr.splitlines() if ln.startswith("step")]
                print(json.dumps(dict(n=n, env=env, rc=r.returncode, wall=time.perf_counter() - t, out=out,
                                      steps=len(steps), last_steps=steps[-3:])), flush=True)
            except subprocess.TimeoutExpired as ex:
                err = (ex.stderr or b"").decode() if isinstance(ex.stderr, bytes) else (ex.stderr or "")
                steps = [ln for ln in err.splitlines() if ln.startswith("step")]
                print(json.dumps(dict(n=n, env=env, timeout=True, steps=len(steps), last_steps=steps[-3:])), flush=True)


if __name__ == "__main__":
    main()
