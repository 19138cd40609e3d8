"""BASELINE config 4 on real TSPLIB instances: gr17 (EXPLICIT,
LOWER_DIAG_ROW), burma14, ulysses16 and ulysses22 (GEO): tests/golden/tsplib/
(data files).

Pinned by the published optimal tour lengths (TSPLIB: burma14 3323,
ulysses16 6859, gr17 2085, ulysses22 7013): the CPU oracle reaches them on
the matrices both readers build (tspgpu.read_tsplib and bin/tsp_search
--tsplib, checked equal), and every GPU path returns the oracle's cost and
tie-broken tour.  The reference itself
cannot read these (Euclidean doubles, <= 16 cities)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
import tspgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TSPLIB = os.path.join(ROOT, "tests", "golden", "tsplib")
BIN = os.path.join(ROOT, "tsp-mpi-reduction_amd", "bin", "tsp_search")
# TSPLIB's published optima
OPTIMUM = {"burma14.tsp": 3323, "ulysses16.tsp": 6859, "gr17.tsp": 2085, "ulysses22.tsp": 7013}


def _matrix(name):
    return tspgpu.read_tsplib(os.path.join(TSPLIB, name))[1]


@pytest.mark.parametrize("name", sorted(OPTIMUM))
def test_oracle_reaches_the_published_optimum(name):
    d = _matrix(name)
    assert d.dtype == np.int32 and (d == d.T).all() and (np.diag(d) == 0).all()
    cost, tour = O.solve_block(d.astype(np.float64))
    assert cost == OPTIMUM[name]
    assert sorted(tour[:-1]) == list(range(d.shape[0])) and tour[0] == tour[-1] == 0
    assert sum(int(d[tour[i], tour[i + 1]]) for i in range(d.shape[0])) == OPTIMUM[name]


@pytest.mark.skipif(not os.path.exists(BIN), reason="bin/tsp_search not built")
@pytest.mark.parametrize("name", sorted(OPTIMUM))
def test_cli_reader_builds_the_same_matrix(name):
    out = subprocess.run([BIN, "--tsplib", os.path.join(TSPLIB, name), "--dump-matrix"], capture_output=True,
                         text=True, timeout=60, check=True).stdout.split()
    n = int(out[0])
    m = np.array([int(x) for x in out[1:]], dtype=np.int32).reshape(n, n)
    assert np.array_equal(m, _matrix(name))


def test_reader_formats_and_distance_functions(tmp_path):
    """EUC_2D / CEIL_2D / ATT on a tiny instance against TSPLIB95's formulas,
    and every EXPLICIT format giving the same matrix."""
    pts = [(0.0, 0.0), (3.0, 4.0), (10.0, 0.5), (7.2, 9.9)]
    body = "".join(f"{i + 1} {x} {y}\n" for i, (x, y) in enumerate(pts))
    import math

    for kind, f in (("EUC_2D", lambda r: int(r + 0.5)), ("CEIL_2D", lambda r: math.ceil(r))):
        p = tmp_path / f"{kind}.tsp"
        p.write_text(f"NAME: t\nDIMENSION: 4\nEDGE_WEIGHT_TYPE: {kind}\nNODE_COORD_SECTION\n{body}EOF\n")
        d = tspgpu.read_tsplib(str(p))[1]
        for i in range(4):
            for j in range(4):
                r = math.dist(pts[i], pts[j])
                assert d[i, j] == (0 if i == j else f(r))
    full = np.array([[0, 5, 9, 4], [5, 0, 3, 8], [9, 3, 0, 6], [4, 8, 6, 0]])
    rows = {
        "FULL_MATRIX": [full[i, j] for i in range(4) for j in range(4)],
        "UPPER_ROW": [full[i, j] for i in range(4) for j in range(i + 1, 4)],
        "LOWER_ROW": [full[i, j] for i in range(4) for j in range(i)],
        "UPPER_DIAG_ROW": [full[i, j] for i in range(4) for j in range(i, 4)],
        "LOWER_DIAG_ROW": [full[i, j] for i in range(4) for j in range(i + 1)],
    }
    for fmt, vals in rows.items():
        p = tmp_path / f"{fmt}.tsp"
        p.write_text(f"NAME: t\nDIMENSION: 4\nEDGE_WEIGHT_TYPE: EXPLICIT\nEDGE_WEIGHT_FORMAT: {fmt}\n"
                     f"EDGE_WEIGHT_SECTION\n{' '.join(map(str, vals))}\nEOF\n")
        assert np.array_equal(tspgpu.read_tsplib(str(p))[1], full), fmt
        if os.path.exists(BIN):
            out = subprocess.run([BIN, "--tsplib", str(p), "--dump-matrix"], capture_output=True, text=True,
                                 timeout=60, check=True).stdout.split()
            assert np.array_equal(np.array(out[1:], dtype=np.int64).reshape(4, 4), full), fmt


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(OPTIMUM))
def test_gpu_paths_match_the_oracle(gpu_ctx, name):
    d = _matrix(name)
    oc, ot = O.solve_block(d.astype(np.float64))
    n = d.shape[0]
    # K2 (integer mode): the prefix-parallel search
    c2, t2, _ = tspgpu.search_solve(gpu_ctx, d)
    assert c2 == int(oc) and t2.tolist() == ot
    # K1-wide on the same integer weights as doubles (exact: small integers)
    cw, tw, _ = gpu_ctx.solve_instance(d.astype(np.float64))
    assert cw == oc and tw.tolist() == ot
    # K1 i32 (the batched kernel; n = 17 runs the extension sizes)
    if n <= tspgpu.MAX_CITIES:
        ci, ti = gpu_ctx.solve_blocks_i32(d[None, :, :])
        assert int(ci[0]) == int(oc) and ti[0][: tspgpu.tour_length(n)].tolist() == ot


@pytest.mark.gpu
@pytest.mark.parametrize("solver", ["k2", "wide", "k1"])
@pytest.mark.parametrize("name", sorted(OPTIMUM))
def test_cli_on_tsplib(name, solver):
    if solver == "k1" and _matrix(name).shape[0] > tspgpu.MAX_CITIES:
        pytest.skip("K1 batch sizes end at MAX_CITIES")
    p = subprocess.run([BIN, "--tsplib", os.path.join(TSPLIB, name), "--solver", solver], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert lines[0].startswith(f"cities {_matrix(name).shape[0]}  mode i32")
    assert float(lines[1].split()[2]) == OPTIMUM[name]
    d = _matrix(name)
    assert [int(x) for x in lines[2].split()[1:]] == O.solve_block(d.astype(np.float64))[1]
