"""K2 host logic, no GPU: the DP tie rule applied to the optimal set O
(tspgpu_select_tour) against the pinned CPU oracle, with O enumerated by brute
force; and the 2-opt upper bound.  Exercised through libtspgpu's C ABI (host
functions only; nothing here launches a kernel).
"""
import itertools

import numpy as np
import pytest

import oracle_py as O
import tspgpu


def left_fold(d, t):
    """tsp.cpp's cost of the closed tour 0, t1..tN, 0 (IEEE double / int)."""
    c = d.dtype.type(0)
    prev = 0
    for x in t:
        c = c + d[prev, x]
        prev = x
    return c + d[prev, 0]


def optimal_set(d):
    """All tours whose left fold equals the optimum (brute force)."""
    n = d.shape[0]
    costs = {}
    for p in itertools.permutations(range(1, n)):
        costs[p] = left_fold(d, p)
    opt = min(costs.values())
    return opt, [p for p, c in costs.items() if c == opt]


def records(opt_set, cost, dtype):
    out = []
    for p in opt_set:
        r = tspgpu.TourRecord()
        r.cost = tspgpu.cost_bits(cost, dtype)
        for i, x in enumerate(p):
            r.city[i] = x
        out.append(r)
    return out


def instances(rng, n, count):
    for k in range(count):
        kind = k % 4
        if kind == 0:
            xy = rng.uniform(0, 1000, size=(n, 2))
        elif kind == 1:
            xy = rng.integers(0, 3, size=(n, 2)).astype(np.float64)  # lattice: heavy ties
        elif kind == 2:
            xy = np.stack([rng.integers(0, 6, size=n), np.zeros(n)], 1).astype(np.float64)  # collinear
        else:
            xy = rng.integers(0, 1000, size=(n, 2)).astype(np.float64)
        cities = [(i, xy[i, 0], xy[i, 1]) for i in range(n)]
        yield O.distance_matrix(cities)


@pytest.mark.parametrize("n", [3, 4, 5, 6, 7, 8])
def test_select_tour_f64_matches_dp(n):
    rng = np.random.default_rng(500 + n)
    for d in instances(rng, n, 24 if n <= 7 else 8):
        opt, oset = optimal_set(d)
        oc, ot = O.solve_block(d)
        assert opt == oc
        tour = tspgpu.select_tour(d, records(oset, opt, tspgpu.F64), opt)
        assert tour.tolist() == ot, (n, len(oset))


@pytest.mark.parametrize("n", [4, 6, 8])
def test_select_tour_i32_matches_dp(n):
    """Integer-matrix extension: symmetric and asymmetric small integers (many
    ties); the oracle runs on the same values as doubles (exact)."""
    rng = np.random.default_rng(900 + n)
    for k in range(16 if n < 8 else 6):
        m = rng.integers(1, 6, size=(n, n)).astype(np.int32)
        if k % 2 == 0:
            m = np.minimum(m, m.T)
        np.fill_diagonal(m, 0)
        opt, oset = optimal_set(m)
        oc, ot = O.solve_block(m.astype(np.float64))
        assert float(opt) == oc
        tour = tspgpu.select_tour(m, records(oset, int(opt), tspgpu.I32), int(opt))
        assert tour.tolist() == ot, (n, k, len(oset))


def test_select_tour_ignores_non_optimal_and_needs_optimal():
    rng = np.random.default_rng(3)
    d = next(instances(rng, 6, 1))
    opt, oset = optimal_set(d)
    worse = [p for p in itertools.permutations(range(1, 6)) if left_fold(d, p) > opt][:5]
    recs = records(oset, opt, tspgpu.F64) + records(worse, opt, tspgpu.F64)  # wrong-cost stragglers
    assert tspgpu.select_tour(d, recs, opt).tolist() == O.solve_block(d)[1]
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.select_tour(d, records(worse, opt, tspgpu.F64), opt)


@pytest.mark.parametrize("n", [5, 9, 16, 24, 32])
def test_heuristic_is_an_upper_bound(n):
    rng = np.random.default_rng(n)
    xy = rng.uniform(0, 1000, size=(n, 2))
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
    cost, tour = tspgpu.heuristic_tour(d)
    assert tour[0] == 0 and tour[-1] == 0 and sorted(tour[1:-1].tolist()) == list(range(1, n))
    assert cost == left_fold(d, tour[1:-1])
    if n <= 16:
        assert cost >= O.solve_block(d)[0]


@pytest.mark.parametrize("n", [6, 17, 30])
def test_heuristic_split_over_ranks_gives_the_same_bound(n):
    """tspgpu_heuristic_tour_starts: W ranks taking the start cities r, r+W, ...
    and the MIN of their costs get exactly the all-starts bound (what
    search_dist.solve_sharded exchanges before the search)."""
    rng = np.random.default_rng(100 + n)
    xy = rng.uniform(0, 1000, size=(n, 2))
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
    full, _ = tspgpu.heuristic_tour(d)
    for W in (1, 2, 3, 8):
        parts = [tspgpu.heuristic_tour(d, first=r, step=W)[0] for r in range(W)]
        assert min(c for c in parts if c is not None) == full
    assert tspgpu.heuristic_tour(d, first=n, step=1) == (None, None)
    di = np.rint(d).astype(np.int32)
    full_i, _ = tspgpu.heuristic_tour(di)
    assert min(tspgpu.heuristic_tour(di, first=r, step=4)[0] for r in range(4)) == full_i


@pytest.mark.parametrize("n", [20, 27, 32])
def test_heuristic_threads_give_the_serial_tour(n, knobs):
    """From 20 cities the multi-start runs on up to 8 host threads
    (TSPGPU_HEURISTIC_THREADS overrides); the results are combined in start
    order, so cost and tour equal the serial run's, f64 and i32."""
    rng = np.random.default_rng(500 + n)
    xy = rng.uniform(0, 1000, size=(n, 2))
    d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
    for m in (d, np.rint(d).astype(np.int32)):
        got = []
        for t in ("1", "3", "8"):
            knobs.set("HEURISTIC_THREADS", t)
            c, tour = tspgpu.heuristic_tour(m)
            got.append((c, tour.tolist()))
        assert got[0] == got[1] == got[2]


def test_search_validation():
    """Host-side argument checks of the K2 entry points (no device needed)."""
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.heuristic_tour(np.zeros((2, 2)))          # n < 3
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.heuristic_tour(np.zeros((33, 33)))        # n > 32
    bad = np.ones((5, 5))
    bad[1, 2] = -1.0
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.heuristic_tour(bad)
    big = np.full((5, 5), 1 << 28, dtype=np.int32)
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.heuristic_tour(big)                       # n * max(d) >= 2^30


# --- device tie rule, host half (tspgpu_tie_key / tspgpu_tie_tour) ----------

def rev_lex(t):
    """tsp()'s tie order among DP-consistent optimal tours: t_N first."""
    return tuple(reversed(t))


@pytest.mark.parametrize("n", [3, 5, 8, 13, 21, 22, 27, 32])
def test_tie_key_orders_reverse_lex_and_round_trips(n):
    """The key is order-isomorphic to reverse-lex order (one u64 up to 20 inner
    cities, a (w0, w1) pair above) and decodes back to the tour."""
    rng = np.random.default_rng(40 + n)
    d = np.ones((n, n))
    np.fill_diagonal(d, 0)
    tours = [rng.permutation(np.arange(1, n)).tolist() for _ in range(60)]
    if n > 3:  # neighbours in reverse-lex order: one swap near the front
        tours += [t[:1] + t[1:2][::-1] + t[2:] for t in tours[:10]]
        tours += [[t[1], t[0]] + t[2:] for t in tours[:10]]
    keys = {}
    for t in tours:
        full = [0] + t + [0]
        k = tspgpu.tie_key(full)
        keys[tuple(t)] = k
        if n - 1 <= 20:
            assert k[1] == 0
        rc, back = tspgpu.tie_tour(d, k[0], k[1], float(n))
        assert rc == 0 and back.tolist() == full  # all-ones: every fold exact
    order_key = sorted(keys, key=lambda t: keys[t])
    order_rl = sorted(keys, key=rev_lex)
    assert order_key == order_rl


@pytest.mark.parametrize("n", [4, 5, 6, 7, 8])
def test_tie_rule_least_key_is_tsp_tour(n):
    """The least key among the optimal tours, once certified, is exactly the
    tour tsp() returns (random, lattice and collinear instances: heavy ties);
    the certificate must hold on most of them."""
    rng = np.random.default_rng(700 + n)
    certified = total = 0
    for d in instances(rng, n, 24 if n <= 7 else 8):
        opt, oset = optimal_set(d)
        best = min(oset, key=lambda p: tspgpu.tie_key([0, *p, 0]))
        assert best == min(oset, key=rev_lex)
        w0, w1 = tspgpu.tie_key([0, *best, 0])
        rc, tour = tspgpu.tie_tour(d, w0, w1, opt)
        total += 1
        if rc == 0:
            certified += 1
            assert tour.tolist() == O.solve_block(d)[1], (n, len(oset))
        else:
            assert rc == -11  # -EAGAIN: the records decide
    assert certified == total  # (the prefix DP proves the cases the one-ulp test cannot)


@pytest.mark.parametrize("n", [4, 6, 8])
def test_tie_rule_integer_costs_always_certified(n):
    rng = np.random.default_rng(990 + n)
    for k in range(12 if n < 8 else 4):
        m = rng.integers(1, 6, size=(n, n)).astype(np.int32)
        if k % 2 == 0:
            m = np.minimum(m, m.T)
        np.fill_diagonal(m, 0)
        opt, oset = optimal_set(m)
        best = min(oset, key=rev_lex)
        w0, w1 = tspgpu.tie_key([0, *best, 0])
        rc, tour = tspgpu.tie_tour(m, w0, w1, int(opt))
        assert rc == 0 and tour.tolist() == O.solve_block(m.astype(np.float64))[1]


def test_tie_tour_rejects_wrong_cost_and_bad_keys():
    rng = np.random.default_rng(8)
    d = next(instances(rng, 7, 1))
    opt, oset = optimal_set(d)
    w0, w1 = tspgpu.tie_key([0, *oset[0], 0])
    assert tspgpu.tie_tour(d, w0, w1, opt * 2)[0] == -22      # -EINVAL: not that cost
    assert tspgpu.tie_tour(d, 10 ** 9, 0, opt)[0] == -22      # digits out of range
    with pytest.raises(tspgpu.TspGpuError):
        tspgpu.tie_key([0, 1, 1, 2, 0])                       # not a permutation


def _needs_prefix_check(d, t):
    """Levels j at which the certificate's one-ulp test fails (a fold one ulp
    below F[j] could round to the same F[j+1]): there it needs G[{t1..tj}][tj]."""
    n = d.shape[0]
    N = n - 1
    F, acc, prev = [0.0] * (N + 2), 0.0, 0
    for j in range(1, N + 1):
        acc = acc + d[prev, t[j]]
        F[j], prev = acc, t[j]
    F[N + 1] = acc + d[prev, 0]
    out = []
    for j in range(2, N + 1):
        dj = d[t[j], t[j + 1]] if j < N else d[t[N], 0]
        if not (np.nextafter(F[j], -np.inf) + dj < F[j + 1]):
            out.append(j)
    return out


@pytest.mark.parametrize("n", [6, 7, 8, 9])
def test_tie_certificate_from_the_optimal_records(n):
    """tspgpu_tie_tour_records (round 6): the certificate's prefix minima from
    the complete optimal set O instead of a Held-Karp DP — with no DP to fall
    back on (ctx None), it must certify exactly what the DP certifies, with
    tsp()'s tour; and a record set missing the winner must not certify where a
    prefix check is needed."""
    rng = np.random.default_rng(4400 + n)
    checked = 0
    for k, d in enumerate(instances(rng, n, 40 if n <= 8 else 12)):
        if k % 4 == 0:  # costs in the thousands: binade crossings along the tour
            d = d * 4.0
        opt, oset = optimal_set(d)
        best = min(oset, key=rev_lex)
        w0, w1 = tspgpu.tie_key([0, *best, 0])
        rc_dp, tour_dp = tspgpu.tie_tour(d, w0, w1, opt)
        recs = records(oset, opt, tspgpu.F64)
        rc, tour = tspgpu.tie_tour_records(None, d, w0, w1, opt, recs)
        assert rc == rc_dp == 0, (n, k, rc, rc_dp)
        assert tour.tolist() == tour_dp.tolist() == O.solve_block(d)[1]
        # (lattice and collinear instances fold exactly: nothing to prove)
        if k % 4 in (0, 3) and _needs_prefix_check(d, [0, *best, 0]):
            checked += 1
            others = [r for r, p in zip(recs, oset) if p != best]
            assert tspgpu.tie_tour_records(None, d, w0, w1, opt, others)[0] == -11  # not the whole O
    assert checked > 0  # (the record path was exercised)
