#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Runs only in the survey container, where /root/reference exists and
`make -C oracle` has compiled it into oracle/_ref/ (ref_harness = the
reference's own tsp.cpp behind a `#define main` harness; tsp = the reference
CLI, run under MPICH's mpirun).  The fixtures are pure data (inputs and the
reference's outputs); nothing of the reference's source is stored.

    python tests/golden/make_golden.py            # rewrite every fixture

Every float is stored twice: exact C99 hex (%a, the value compared) and
%.17g (for humans).
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
HARNESS = os.path.join(REF, "ref_harness")
REF_TSP = os.path.join(REF, "tsp")
MPIRUN = "/opt/conda/bin/mpirun"


def harness(*args: str) -> list[list[str]]:
    out = subprocess.run([HARNESS, *args], check=True, capture_output=True, text=True).stdout
    return [ln.split() for ln in out.splitlines() if ln[:2] in ("S ", "C ", "D ", "F ")]


def parse_solutions(rows):
    sols = []
    for r in rows:
        length = int(r[4])
        sols.append({"cost_hex": r[2], "cost": r[3], "ids": [int(x) for x in r[5:5 + length]]})
    return sols


def gen_seed0_blocks():
    """tsp() on the reference's own generated instances (srand(0), tsp.cpp:273)."""
    cases = []
    for n in range(2, 17):
        cases.append((n, 1, 1000, 1000))
    cases += [(16, 1, 1, 1), (4, 2, 0, 0), (5, 7, 500, 500), (6, 8, 1000, 1000), (7, 9, 800, 600),
              (8, 12, 1000, 1000), (10, 6, 500, 500), (12, 4, 1000, 1000), (14, 4, 1000, 1000),
              (16, 3, 1000, 1000), (3, 5, 10, 10), (9, 10, 7, 3)]
    out = []
    for (n, B, X, Y) in cases:
        cities = harness("gen", str(n), str(B), str(X), str(Y))
        sols = parse_solutions(harness("solve", str(n), str(B), str(X), str(Y)))
        blocks = [[] for _ in range(B)]
        for r in cities:
            blocks[int(r[1])].append([int(r[2]), r[3], r[4]])
        out.append({"n": n, "B": B, "X": X, "Y": Y, "cities": blocks, "solutions": sols})
        print(f"seed0 n={n} B={B} X={X} Y={Y}: {[s['cost'] for s in sols][:3]}", flush=True)
    return out


def gen_dist():
    out = []
    for (n, B, X, Y) in [(16, 1, 1000, 1000), (8, 4, 1000, 1000), (12, 2, 123, 4567)]:
        d = {}
        for r in harness("dist", str(n), str(B), str(X), str(Y)):
            d.setdefault(int(r[1]), [[None] * n for _ in range(n)])[int(r[2])][int(r[3])] = r[4]
        out.append({"n": n, "B": B, "X": X, "Y": Y, "dist_hex": [d[b] for b in range(B)]})
    return out


def write_blockfile(path, blocks):
    with open(path, "w") as f:
        for blk in blocks:
            f.write(f"B {len(blk)}\n")
            for (cid, x, y) in blk:
                f.write(f"{cid} {float(x).hex()} {float(y).hex()}\n")


def gen_file_instances(name, blocks, chunk=64):
    """tsp() on externally supplied city lists (tie-heavy and random inputs)."""
    tmp = os.path.join(REF, f"_{name}.txt")
    sols = []
    for i in range(0, len(blocks), chunk):
        write_blockfile(tmp, blocks[i:i + chunk])
        sols += parse_solutions(harness("solvefile", tmp))
    os.remove(tmp)
    return [{"cities": [[c, float(x).hex(), float(y).hex()] for (c, x, y) in blk], "solution": s}
            for blk, s in zip(blocks, sols)]


def tie_instances():
    rng = np.random.default_rng(20261015)
    blocks = []
    # collinear integer cities (every tour and its reverse tie; many optima tie)
    for n in range(3, 12):
        for _ in range(12):
            xs = rng.integers(0, 6, size=n)
            blocks.append([(i, float(xs[i]), 0.0) for i in range(n)])
    # small-integer lattice (heavy ties, coincident cities)
    for n in range(3, 13):
        for _ in range(10):
            xs = rng.integers(0, 3, size=n)
            ys = rng.integers(0, 3, size=n)
            blocks.append([(100 + i, float(xs[i]), float(ys[i])) for i in range(n)])
    # all cities coincident
    for n in (3, 6, 9, 13):
        blocks.append([(i, 5.0, 5.0) for i in range(n)])
    # regular polygon-ish integer points
    for n in (8, 12, 14):
        blocks.append([(i, float(round(100 * np.cos(2 * np.pi * i / n))), float(round(100 * np.sin(2 * np.pi * i / n))))
                       for i in range(n)])
    return blocks


def random_instances():
    rng = np.random.default_rng(424242)
    blocks = []
    for n in range(3, 14):
        for _ in range(16 if n <= 11 else 6):
            xy = rng.uniform(0, 1000, size=(n, 2))
            blocks.append([(7 * i + 3, float(xy[i, 0]), float(xy[i, 1])) for i in range(n)])
    # clustered (config-4 style substitute), a few at n=14..16
    for n, cnt in ((14, 3), (15, 2), (16, 2)):
        for _ in range(cnt):
            centers = rng.uniform(0, 1000, size=(4, 2))
            lab = rng.integers(0, 4, size=n)
            xy = centers[lab] + rng.normal(0, 50, size=(n, 2))
            blocks.append([(i, float(xy[i, 0]), float(xy[i, 1])) for i in range(n)])
    return blocks


def k1_batch_instances(n, count, seed):
    """Batches for K1's large-batch kernel (variant 5 at n = 13..16): a third
    on the 0..3 lattice (coincident cities, tie storms), a third on the 0..39
    lattice (many tied optima), a third uniform doubles in [0, 1000)."""
    rng = np.random.default_rng(seed)
    blocks = []
    for b in range(count):
        kind = b % 3
        if kind == 0:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)
        elif kind == 1:
            xy = rng.integers(0, 40, size=(n, 2)).astype(np.float64)
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        blocks.append([(1000 * b + i, float(xy[i, 0]), float(xy[i, 1])) for i in range(n)])
    return blocks


def gen_k1_batches(count=522, workers=8):
    """tsp() (the reference, -O0) on 522 blocks at each of n = 13..16, solved
    in parallel harness processes (chunks of 6 blocks)."""
    from concurrent.futures import ThreadPoolExecutor

    out = []
    for n in (13, 14, 15, 16):
        blocks = k1_batch_instances(n, count, 20261017 + n)
        chunks = [blocks[i:i + 6] for i in range(0, len(blocks), 6)]

        def solve(ci):
            tmp = os.path.join(REF, f"_k1b_{n}_{ci}.txt")
            write_blockfile(tmp, chunks[ci])
            try:
                return parse_solutions(harness("solvefile", tmp))
            finally:
                os.remove(tmp)

        with ThreadPoolExecutor(workers) as ex:
            sols = [s for part in ex.map(solve, range(len(chunks))) for s in part]
        assert len(sols) == len(blocks)
        rows = []
        for blk, s in zip(blocks, sols):
            xy = [[c[1], c[2]] for c in blk]
            integral = all(v == int(v) for p in xy for v in p)
            rows.append({"id0": blk[0][0], "xy": [[int(a), int(b)] for a, b in xy] if integral
                         else [[float(a).hex(), float(b).hex()] for a, b in xy],
                         "cost_hex": s["cost_hex"], "ids": s["ids"]})
        out.append({"n": n, "blocks": rows})
        print(f"k1 batch n={n}: {len(rows)} blocks", flush=True)
    return out


def gen_fold():
    out = []
    for (n, B, X, Y) in [(5, 7, 500, 500), (6, 8, 1000, 1000), (8, 12, 1000, 1000), (4, 16, 1000, 1000), (3, 5, 100, 100)]:
        rows = harness("fold", str(n), str(B), str(X), str(Y))
        out.append({"n": n, "B": B, "X": X, "Y": Y, "steps": parse_solutions(rows)})
    return out


FINAL_RE = re.compile(r"^TSP ran in (\d+) ms for (\d+) cities and the trip cost (.*)$")


def run_cli(args, P):
    cmd = [MPIRUN, "-np", str(P), REF_TSP, *args] if P > 0 else [REF_TSP, *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    lines = p.stdout.splitlines()
    norm = [FINAL_RE.sub(lambda m: f"TSP ran in <ms> ms for {m.group(2)} cities and the trip cost {m.group(3)}", ln)
            for ln in lines]
    return {"rc": p.returncode, "lines": norm}


def gen_cli():
    cases = []
    mat = {
        (6, 4, 1000, 1000): range(1, 5),
        (6, 8, 1000, 1000): range(1, 9),
        (8, 12, 1000, 1000): range(1, 9),
        (5, 7, 500, 500): range(1, 8),
        (10, 16, 1000, 1000): range(1, 9),
        (7, 9, 800, 600): range(1, 9),
        (12, 4, 1000, 1000): (4,),
        (10, 6, 500, 500): (3,),
        (4, 256, 1000, 1000): (1, 8),
        (16, 1, 1000, 1000): (1,),
        (16, 1, 1, 1): (1,),
        (4, 2, 0, 0): (1,),
        (3, 30, 1000, 1000): (1, 3, 6),
        (11, 5, 1000, 1000): (5,),
        (9, 32, 1000, 1000): (8,),
        # SURVEY Appendix B's 16-city multi-block runs (the reference's own
        # strong-scaling axis): one fixed B over P ranks
        (16, 8, 1000, 1000): (1, 2, 4, 8),
        (16, 16, 1000, 1000): (8,),
        (14, 64, 1000, 1000): (8,),
    }
    for (n, B, X, Y), Ps in mat.items():
        for P in Ps:
            r = run_cli([str(n), str(B), str(X), str(Y)], P)
            cases.append({"args": [n, B, X, Y], "P": P, **r})
            print(f"cli {n} {B} {X} {Y} P={P}: {r['lines'][-1] if r['lines'] else r}", flush=True)
    # argument errors (P=1, no mpirun)
    for args in (["17", "1", "1000", "1000"], ["4", "1", "1000"], []):
        r = run_cli(args, 0)
        cases.append({"args": args, "P": 1, "error_case": True, **r})
    return cases


def gen_cli_large():
    """SURVEY Appendix B's merge-dominated runs (mergeBlocks, tsp.cpp:202-269, is
    O(L1*L2^2) there): minutes of reference CPU time each, so they live in their
    own fixture (cli_large.json) and are regenerated only on request."""
    cases = []
    for (n, B, X, Y), Ps in {(4, 1024, 1000, 1000): (1, 8), (8, 1024, 1000, 1000): (8,)}.items():
        for P in Ps:
            r = run_cli([str(n), str(B), str(X), str(Y)], P)
            cases.append({"args": [n, B, X, Y], "P": P, **r})
            print(f"cli {n} {B} {X} {Y} P={P}: {r['lines'][-1] if r['lines'] else r}", flush=True)
    return cases


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference first: make -C oracle (needs /root/reference)")
    # cli_large (~10 min of reference time) runs only when named
    which = set(sys.argv[1:]) or {"seed0", "dist", "ties", "random", "fold", "cli", "k1batch"}
    jobs = {
        "seed0": ("seed0_blocks.json", gen_seed0_blocks),
        "dist": ("seed0_dist.json", gen_dist),
        "ties": ("tie_blocks.json", lambda: gen_file_instances("ties", tie_instances())),
        "random": ("random_blocks.json", lambda: gen_file_instances("random", random_instances())),
        "fold": ("fold.json", gen_fold),
        "cli": ("cli.json", gen_cli),
        "k1batch": ("k1_batches.json", gen_k1_batches),
        "cli_large": ("cli_large.json", gen_cli_large),
    }
    for key in sorted(which):
        fname, fn = jobs[key]
        data = {"generator": "tests/golden/make_golden.py", "source": "reference compiled from /root/reference "
                "(oracle/Makefile, -O0, MPICH 3.3.2, glibc 2.35)", "data": fn()}
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(data, f, separators=(",", ":"))
        print("wrote", fname, flush=True)


if __name__ == "__main__":
    main()
