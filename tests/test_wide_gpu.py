"""K1-wide (csrc/hkwide.hip): one instance's Held-Karp over the whole GPU.
Same bits and tour as the reference (goldens), the oracle and K1; past K1's
sizes (n = 21, 22) it must agree with K2, an independent exact algorithm."""
import numpy as np
import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu


def test_seed0_fixtures(gpu_ctx):
    for case in O.load_golden("seed0_blocks.json"):
        if case["n"] < 3:
            continue
        for blk, sol in zip(case["cities"], case["solutions"]):
            cities = [(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in blk]
            d = tspgpu.distance_matrix([cities])[0]
            cost, tour, _ = gpu_ctx.solve_instance(d)
            assert cost == O.hexf(sol["cost_hex"]) and [cities[t][0] for t in tour] == sol["ids"]


@pytest.mark.parametrize("name", ["tie_blocks.json", "random_blocks.json"])
def test_file_fixtures(gpu_ctx, name):
    for inst in O.load_golden(name):
        cities = [(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in inst["cities"]]
        if len(cities) < 3:
            continue
        d = tspgpu.distance_matrix([cities])[0]
        cost, tour, _ = gpu_ctx.solve_instance(d)
        assert cost == O.hexf(inst["solution"]["cost_hex"])
        assert [cities[t][0] for t in tour] == inst["solution"]["ids"]


@pytest.mark.parametrize("n", [3, 6, 10, 14, 17, 20])
def test_against_oracle_and_k1(gpu_ctx, n):
    rng = np.random.default_rng(300 + n)
    for k in range(4 if n < 17 else 2):
        xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64) if k % 2 else rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, _ = gpu_ctx.solve_instance(d)
        oc, ot = O.solve_block(d)
        assert cost == oc and tour.tolist() == ot
        c1, t1 = gpu_ctx.solve_blocks(d[None])
        assert c1[0] == cost and t1[0].tolist() == tour.tolist()


@pytest.mark.parametrize("n", [21, 22])
def test_beyond_k1_agrees_with_k2(gpu_ctx, n):
    rng = np.random.default_rng(n)
    xy = rng.uniform(0, 1000, size=(n, 2))
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
    cost, tour, _ = gpu_ctx.solve_instance(d)
    c2, t2, _ = tspgpu.search_solve(gpu_ctx, d)
    assert cost == c2 and tour.tolist() == t2.tolist()


def test_rejects_bad_input(gpu_ctx):
    with pytest.raises(tspgpu.TspGpuError):
        gpu_ctx.solve_instance(np.zeros((32, 32)))
    bad = np.ones((5, 5))
    bad[0, 1] = np.nan
    with pytest.raises(tspgpu.TspGpuError):
        gpu_ctx.solve_instance(bad)


@pytest.mark.parametrize("form", ["0", "1"])
def test_push_and_pull_forms(gpu_ctx, form, knobs):
    """Both layer forms (row-owner push, per-destination pull) on the goldens
    (tie-heavy included) and on random / lattice instances vs the oracle."""
    knobs.set("WIDE_PULL", form)
    for inst in O.load_golden("tie_blocks.json"):
        cities = [(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in inst["cities"]]
        if len(cities) < 3:
            continue
        d = tspgpu.distance_matrix([cities])[0]
        cost, tour, _ = gpu_ctx.solve_instance(d)
        assert cost == O.hexf(inst["solution"]["cost_hex"])
        assert [cities[t][0] for t in tour] == inst["solution"]["ids"]
    rng = np.random.default_rng(int(form) + 77)
    for n in (3, 5, 9, 13, 16, 18, 20):
        for lattice in (False, True):
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64) if lattice else rng.uniform(0, 1000, size=(n, 2))
            d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
            cost, tour, _ = gpu_ctx.solve_instance(d)
            oc, ot = O.solve_block(d)
            assert cost == oc and tour.tolist() == ot, (form, n, lattice)
