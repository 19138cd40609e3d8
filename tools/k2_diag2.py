"""Reproduce a failing K2 case under several settings (development aid)."""
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
d = np.asarray(k2_instance(32, 35))
try:
    t = time.perf_counter()
    c, tour, st = tspgpu.search_solve(ctx, d)
    print(json.dumps(dict(ok=True, ms=(time.perf_counter() - t) * 1e3, cost=c, st={{k: st[k] for k in ("records", "phases", "fallback", "tie", "rounds", "nodes", "kernel_ms")}})))
except Exception as ex:
    print(json.dumps(dict(ok=False, err=str(ex))))
'''


def main():
    for env in ({"TSPGPU_SEARCH_MST": "0"}, {"TSPGPU_SEARCH_MST": "0", "TSPGPU_SEARCH_TIE": "0"},
                {"TSPGPU_SEARCH_MST": "0", "TSPGPU_CHAIN_MAXN": "32"}):
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)],
                           env=dict(os.environ, TSPGPU_SEARCH_DEBUG="2", **env), capture_output=True, text=True, timeout=100)
        err = [ln for ln in r.stderr.splitlines() if not ln.startswith("step")]
        steps = [ln for ln in r.stderr.splitlines() if ln.startswith("step")]
        print(json.dumps(dict(env=env, out=r.stdout.strip()[-600:], err=err[-5:], steps=len(steps), first=steps[:3],
                              last=steps[-2:])), flush=True)


if __name__ == "__main__":
    main()
