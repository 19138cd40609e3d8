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


def _host_reduce(sols, P):
    B, L = len(sols), len(sols[0][0])
    flat = (tspgpu.City * (B * L))()
    costs = (ctypes.c_double * B)()
    for b, (path, cost) in enumerate(sols):
        costs[b] = cost
        for i, (cid, x, y) in enumerate(path):
            flat[b * L + i].id, flat[b * L + i].x, flat[b * L + i].y = cid, x, y
    final = ctypes.c_double()
    log = ctypes.create_string_buffer(1 << 16)
    assert H.tsphost_reduce(flat, L, costs, B, P, ctypes.byref(final), log, len(log)) == 0
    return final.value, log.value.decode()


@pytest.mark.parametrize("kind,n,B,P", [("lattice", 6, 48, 1), ("lattice", 9, 40, 3), ("random", 8, 300, 8),
                                        ("random", 5, 1100, 1)])
def test_persistent_fold_matches_host(gpu_ctx, knobs, kind, n, B, P):
    """The per-rank persistent fold (fold_persist_kernel, one launch for every
    rank's fold) against the host replay and against the per-merge kernels:
    tie-heavy lattice blocks (near-tied candidates stall a rank: the host
    merges exactly and the kernel resumes), random blocks over 8 ranks, and a
    fold that outgrows the 4096-city LDS path (4 x 1100 cities at P = 1: the
    per-merge kernels finish it)."""
    rng = np.random.default_rng(n * 1000 + B + P)
    blocks = []
    for b in range(B):
        xy = (rng.integers(0, 3, size=(n, 2)) + 3 * np.array([b % 7, b // 7])).astype(np.float64) \
            if kind == "lattice" else rng.uniform(0, 1000, size=(n, 2))
        blocks.append([(b * n + i, xy[i, 0], xy[i, 1]) for i in range(n)])
    sols = _solve_all(blocks)
    hf, hlog = _host_reduce(sols, P)
    paths, costs = [p for p, _ in sols], [c for _, c in sols]
    f1, log1 = gpu_ctx.reduce(paths, costs, P)
    knobs.set("K3_PERSIST", "0")
    f0, log0 = gpu_ctx.reduce(paths, costs, P)
    assert f1 == hf and f0 == hf, (f1, f0, hf)
    assert log1 == log0 and sorted(log1.splitlines()) == sorted(hlog.splitlines())
