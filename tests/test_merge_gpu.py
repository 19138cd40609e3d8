"""K3 (csrc/merge.hip): the reference's mergeBlocks and reduction tree with
the paths on the GPU, through the C ABI, against the reference's own fold
steps and mpirun output (goldens) and the host parity layer."""
import ctypes
import re

import numpy as np
import pytest

import oracle_py as O
import tspgpu
from test_host import H, _solve_all, city_array, generate

pytestmark = pytest.mark.gpu
FINAL = re.compile(r"trip cost (\S+)$")


def host_merge(p1, c1, p2, c2):
    a1, a2 = city_array(p1), city_array(p2)
    out = (tspgpu.City * (len(a1) + len(a2)))()
    cost = ctypes.c_double()
    L = H.tsphost_merge(a1, len(a1), c1, a2, len(a2), c2, out, ctypes.byref(cost))
    if L < 0:
        return None, None
    return [(out[j].id, out[j].x, out[j].y) for j in range(L)], cost.value


@pytest.mark.parametrize("case", O.load_golden("fold.json"), ids=lambda c: f"n{c['n']}B{c['B']}")
def test_fold_matches_reference(gpu_ctx, case):
    sols = _solve_all(generate(case["n"], case["B"], case["X"], case["Y"]))
    acc_path, acc_cost = sols[0]
    for i, st in enumerate(case["steps"]):
        if i:
            acc_path, acc_cost = gpu_ctx.merge(acc_path, acc_cost, *sols[i])
        assert acc_cost == O.hexf(st["cost_hex"])
        assert [c[0] for c in acc_path] == st["ids"]


CLI = [c for c in O.load_golden("cli.json") if not c.get("error_case")]


@pytest.mark.parametrize("case", CLI, ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_reduce_matches_mpirun(gpu_ctx, case):
    n, B, X, Y = case["args"]
    sols = _solve_all(generate(n, B, X, Y))
    final, log = gpu_ctx.reduce([p for p, _ in sols], [c for _, c in sols], case["P"])
    assert "%f" % final == FINAL.search(case["lines"][-1]).group(1)
    assert sorted(log.splitlines()) == sorted(ln for ln in case["lines"] if ln.startswith("process "))


def _random_path(rng, n, start_id, kind):
    if kind == "lattice":
        xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)
    elif kind == "dup":
        xy = np.repeat(rng.uniform(0, 1000, size=((n + 1) // 2, 2)), 2, axis=0)[:n]
    else:
        xy = rng.uniform(0, 1000, size=(n, 2))
    cities = [(start_id + i, xy[i, 0], xy[i, 1]) for i in range(n)]
    return cities + [cities[0]], float(rng.uniform(100, 5000))


@pytest.mark.parametrize("kind", ["random", "lattice", "dup"])
def test_merge_matches_host(gpu_ctx, kind):
    """Random, tie-heavy (lattice) and duplicated-city paths, growing folds."""
    rng = np.random.default_rng({"random": 1, "lattice": 2, "dup": 3}[kind])
    acc, acc_c = _random_path(rng, 9, 0, kind)
    hacc, hacc_c = acc, acc_c
    for step in range(40):
        p2, c2 = _random_path(rng, int(rng.integers(2, 17)), 1000 * (step + 1), kind)
        if len(p2) == 3:  # the n = 2 quirk: a 2-city "tour" without the closing city
            p2 = p2[1:]
        hres, hcost = host_merge(hacc, hacc_c, p2, c2)
        if hres is None:
            with pytest.raises(tspgpu.TspGpuError) as e:
                gpu_ctx.merge(acc, acc_c, p2, c2)
            assert e.value.code == -35  # -EDEADLK: the reference loops forever here
            continue
        acc, acc_c = gpu_ctx.merge(acc, acc_c, p2, c2)
        hacc, hacc_c = hres, hcost
        assert acc_c == hacc_c and [c[0] for c in acc] == [c[0] for c in hacc], step


def test_large_merge_matches_host(gpu_ctx):
    """A 20k-city running path against a block: the GPU search at scale."""
    rng = np.random.default_rng(8)
    p1, c1 = _random_path(rng, 20000, 0, "random")
    p2, c2 = _random_path(rng, 16, 10 ** 6, "random")
    g, gc = gpu_ctx.merge(p1, c1, p2, c2)
    h, hc = host_merge(p1, c1, p2, c2)
    assert gc == hc and [c[0] for c in g] == [c[0] for c in h]
