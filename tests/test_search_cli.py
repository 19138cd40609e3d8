"""bin/tsp_search — the single-instance front end (K2 over 1..G GPUs with an
RCCL all-reduce of the incumbent) and its extension inputs: seeded random and
clustered cities (configs 4/5 stand-ins), TSPLIB-style coordinate files, and
integer distance matrices (config 1).  Answers are checked against the pinned
CPU oracle (f64: the reference's own distances; integers: exact)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
import tspgpu

BIN = os.path.join(os.path.dirname(tspgpu.TSP_BIN), "tsp_search")


def run(*args, timeout=300):
    p = subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout, p.stderr


def parse(out):
    cost = tour = None
    for ln in out.splitlines():
        if ln.startswith("optimal cost "):
            cost = float(ln.split()[2])
        if ln.startswith("tour "):
            tour = [int(x) for x in ln.split()[1:]]
    return cost, tour


def test_usage_and_input_errors(tmp_path):
    assert run("--bogus")[0] == 1
    assert run()[0] == 2                                   # no instance
    assert run("--random", "40")[0] == 2                   # > 32 cities
    bad = tmp_path / "m.txt"
    bad.write_text("4\n0 1 2\n")
    assert run("--matrix", bad)[0] == 2                    # short matrix
    assert run("--cities", tmp_path / "missing.tsp")[0] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("--random", 12, "--seed", 3), ("--random", 16, "--seed", 7),
                                  ("--random", 16, "--clustered", 4, "--seed", 1),
                                  ("--random", 18, "--seed", 2)])
def test_random_instances_verify_against_k1(args):
    rc, out, err = run(*args, "--solver", "k2", "--verify")
    assert rc == 0, err
    assert "K1 check: identical cost and tour" in out


@pytest.mark.gpu
def test_tsplib_file_and_rounding(tmp_path):
    rng = np.random.default_rng(17)
    xy = rng.uniform(0, 1000, size=(14, 2))
    text = "NAME : synth14\nTYPE : TSP\nDIMENSION : 14\nEDGE_WEIGHT_TYPE : EUC_2D\nNODE_COORD_SECTION\n"
    text += "".join(f"{i + 1} {float(x)!r} {float(y)!r}\n" for i, (x, y) in enumerate(xy)) + "EOF\n"
    f = tmp_path / "synth14.tsp"
    f.write_text(text)
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(14)])
    for solver in ("k1", "k2"):
        rc, out, err = run("--cities", f, "--solver", solver)
        assert rc == 0, err
        assert parse(out) == O.solve_block(d)
    rc, out, err = run("--cities", f, "--tsplib-round", "--solver", "k2")
    assert rc == 0, err
    di = np.rint(d)
    oc, ot = O.solve_block(di)
    assert parse(out) == (oc, ot)


@pytest.mark.gpu
@pytest.mark.parametrize("n,hi,sym", [(12, 1000, True), (12, 6, True), (14, 1000, False)])
def test_integer_matrix(tmp_path, n, hi, sym):
    """Config 1: an integer distance matrix (symmetric or not, few or many ties)."""
    rng = np.random.default_rng(n * hi)
    m = rng.integers(1, hi, size=(n, n))
    if sym:
        m = np.minimum(m, m.T)
    np.fill_diagonal(m, 0)
    f = tmp_path / "m.txt"
    f.write_text(f"{n}\n" + "\n".join(" ".join(map(str, r)) for r in m) + "\n")
    rc, out, err = run("--matrix", f, "--solver", "k2", "--verify")
    assert rc == 0, err
    assert "mode i32" in out
    assert parse(out) == O.solve_block(m.astype(np.float64))


@pytest.mark.gpu
def test_coincident_cities_fall_back_to_k1(tmp_path):
    f = tmp_path / "z.txt"
    f.write_text("13\n" + "\n".join(" ".join("0.0" for _ in range(13)) for _ in range(13)) + "\n")
    rc, out, err = run("--matrix", f, "--solver", "k2")
    assert rc == 0, err
    assert parse(out) == O.solve_block(np.zeros((13, 13)))


@pytest.mark.gpu
def test_rccl_path_with_one_gpu():
    """--gpus 1 with K2 (the all-reduce is skipped for a single GPU), auto
    (K1-wide) and wide beyond K1's 20 cities, checked against K2."""
    res = {}
    for solver in ("k2", "auto", "k1"):
        rc, out, err = run("--random", 13, "--seed", 9, "--solver", solver, "--verify")
        assert rc == 0, err
        assert ("solver wide" in out) == (solver == "auto")
        res[solver] = parse(out)
    assert res["k2"] == res["auto"] == res["k1"]
    rc, out, err = run("--random", 23, "--seed", 4, "--solver", "wide")
    assert rc == 0, err
    rc2, out2, err2 = run("--random", 23, "--seed", 4, "--solver", "k2")
    assert rc2 == 0, err2
    assert parse(out) == parse(out2)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [("--random", 11, "--seed", 5), ("--random", 12, "--clustered", 3, "--seed", 2)])
def test_enum_solver_matches_k1(args):
    """--solver enum: every (n-1)! tour enumerated on GPU 0 (config 2's
    exhaustive mode); same cost and tie-broken tour as K1 (--verify)."""
    rc, out, err = run(*args, "--solver", "enum", "--verify")
    assert rc == 0, err
    assert "K1 check: identical cost and tour" in out
    assert "search nodes" in out
