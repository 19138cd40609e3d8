"""ctypes view of oracle/liboracle.so — the CPU checker.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (libtspgpu / the `tsp` binary) never does.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


class OracleCity(ctypes.Structure):
    _fields_ = [("id", ctypes.c_int), ("x", ctypes.c_double), ("y", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-C", ORACLE_DIR, "liboracle.so"], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        cp = ctypes.POINTER(OracleCity)
        L.oracle_distance_matrix.argtypes = [cp, ctypes.c_int, dp]
        L.oracle_solve_block.argtypes = [dp, ctypes.c_int, dp, ip]
        L.oracle_solve_block.restype = ctypes.c_int
        L.oracle_generate.argtypes = [ctypes.c_int] * 4 + [cp]
        L.oracle_distribution_counts.argtypes = [ctypes.c_int, ctypes.c_int, ip]
        L.oracle_blocks_per_dim.argtypes = [ctypes.c_int, ip, ip]
        L.oracle_merge_blocks.argtypes = [cp, ctypes.c_int, ctypes.c_double, cp, ctypes.c_int, ctypes.c_double, cp, dp]
        L.oracle_merge_blocks.restype = ctypes.c_int
        L.oracle_pipeline.argtypes = [ctypes.c_int] * 5 + [dp, ctypes.c_char_p, ctypes.c_int]
        L.oracle_pipeline.restype = ctypes.c_int
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def cities_array(cities):
    """cities: iterable of (id, x, y) -> ctypes array of OracleCity."""
    cities = list(cities)
    arr = (OracleCity * len(cities))()
    for i, (cid, x, y) in enumerate(cities):
        arr[i].id, arr[i].x, arr[i].y = int(cid), float(x), float(y)
    return arr


def distance_matrix(cities) -> np.ndarray:
    arr = cities_array(cities)
    n = len(arr)
    d = np.zeros((n, n), dtype=np.float64)
    lib().oracle_distance_matrix(arr, n, _dp(d))
    return d


def solve_block(d: np.ndarray):
    """-> (cost, tour list of local indices)"""
    d = np.ascontiguousarray(d, dtype=np.float64)
    n = d.shape[0]
    cost = ctypes.c_double()
    tour = np.zeros(n + 1, dtype=np.int32)
    L = lib().oracle_solve_block(_dp(d), n, ctypes.byref(cost), tour.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    if L < 0:
        raise ValueError("oracle_solve_block failed")
    return cost.value, tour[:L].tolist()


def generate(n, B, X, Y):
    """-> list of B blocks, each a list of (id, x, y)"""
    arr = (OracleCity * (n * B))()
    lib().oracle_generate(n, B, X, Y, arr)
    return [[(arr[b * n + j].id, arr[b * n + j].x, arr[b * n + j].y) for j in range(n)] for b in range(B)]


def distribution_counts(B, P):
    cnt = np.zeros(P, dtype=np.int32)
    lib().oracle_distribution_counts(B, P, cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return cnt.tolist()


def merge_blocks(p1, c1, p2, c2):
    a1, a2 = cities_array(p1), cities_array(p2)
    out = (OracleCity * (len(a1) + len(a2)))()
    cost = ctypes.c_double()
    L = lib().oracle_merge_blocks(a1, len(a1), c1, a2, len(a2), c2, out, ctypes.byref(cost))
    if L < 0:
        raise ValueError("merge does not terminate in the reference")
    return [(out[i].id, out[i].x, out[i].y) for i in range(L)], cost.value


def pipeline(n, B, X, Y, P):
    cost = ctypes.c_double()
    buf = ctypes.create_string_buffer(1 << 16)
    rc = lib().oracle_pipeline(n, B, X, Y, P, ctypes.byref(cost), buf, len(buf))
    if rc != 0:
        raise ValueError("pipeline undefined in the reference for these arguments")
    return cost.value, buf.value.decode()


def load_golden(name):
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return json.load(f)["data"]


def hexf(s: str) -> float:
    return float.fromhex(s)


def k1_batch_blocks(case):
    """City lists of one n of tests/golden/k1_batches.json (lattice coordinates
    stored as integers, uniform ones as C99 hex)."""
    out = []
    for blk in case["blocks"]:
        conv = (lambda v: float(v)) if isinstance(blk["xy"][0][0], int) else hexf
        out.append([(blk["id0"] + i, conv(x), conv(y)) for i, (x, y) in enumerate(blk["xy"])])
    return out
