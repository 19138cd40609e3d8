"""K2 (prefix-parallel exact search of one instance, csrc/search.hip) on the
GPU through the C ABI: the same cost bits and the same tour as the reference's
tsp() (goldens) and the pinned oracle, f64 and the integer-matrix extension,
one GPU and sharded.

Run on an MI355X:  python -m pytest tests -m gpu
"""
import numpy as np
import pytest

import oracle_py as O
import search_dist
import tspgpu

pytestmark = pytest.mark.gpu


def _cities(case_cities):
    return [(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in case_cities]


def test_seed0_fixtures(gpu_ctx):
    """The reference's own instances (./tsp n B 1000 1000, n = 3..16): golden cost and tour."""
    for case in O.load_golden("seed0_blocks.json"):
        if case["n"] < 3:
            continue
        for blk, sol in zip(case["cities"], case["solutions"]):
            cities = _cities(blk)
            d = tspgpu.distance_matrix([cities])[0]
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            assert cost == O.hexf(sol["cost_hex"]), (case["n"], st)
            assert [cities[t][0] for t in tour] == sol["ids"], (case["n"], st)


@pytest.mark.parametrize("name", ["tie_blocks.json", "random_blocks.json"])
def test_file_fixtures(gpu_ctx, name):
    """Tie-heavy (collinear, lattice, coincident cities) and random goldens."""
    for inst in O.load_golden(name):
        cities = _cities(inst["cities"])
        if len(cities) < 3:
            continue
        d = tspgpu.distance_matrix([cities])[0]
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        assert cost == O.hexf(inst["solution"]["cost_hex"]), (name, len(cities), st)
        assert [cities[t][0] for t in tour] == inst["solution"]["ids"], (name, len(cities), st)


@pytest.mark.parametrize("n", [3, 4, 5, 7, 9, 11, 13, 15, 16, 17, 18, 20])
def test_f64_against_oracle(gpu_ctx, n):
    rng = np.random.default_rng(4000 + n)
    for k in range(6 if n <= 14 else 2):
        if k % 3 == 1:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)  # lattice ties
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        oc, ot = O.solve_block(d)
        assert cost == oc, (n, k, st)
        assert tour.tolist() == ot, (n, k, st)


@pytest.mark.parametrize("n", [13, 16, 19])
def test_device_bound_against_host_bound(gpu_ctx, n, knobs):
    """search_solve below 20 cities takes its initial bound from the device
    heuristic in the init launch (search.hip init_heuristic): same answers as
    with the host heuristic's bound (knob SEARCH_DEVICE_BOUND=0) and as the
    oracle, on f64 points, lattice ties and asymmetric integer matrices."""
    rng = np.random.default_rng(9100 + n)
    for k in range(3):
        if k == 0:
            xy = rng.uniform(0, 1000, size=(n, 2))
            d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        elif k == 1:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)
            d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        else:
            d = rng.integers(1, 1000, size=(n, n)).astype(np.int32)
            np.fill_diagonal(d, 0)
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        knobs.set("SEARCH_DEVICE_BOUND", 0)
        hcost, htour, hst = tspgpu.search_solve(gpu_ctx, d)
        knobs.clear("SEARCH_DEVICE_BOUND")
        assert cost == hcost and tour.tolist() == htour.tolist(), (n, k)
        if n <= 16:
            oc, ot = O.solve_block(np.asarray(d, dtype=np.float64))
            assert float(cost) == oc and tour.tolist() == ot, (n, k)


@pytest.mark.parametrize("n", [4, 8, 12, 14, 16, 18])
def test_i32_against_oracle(gpu_ctx, n):
    """Integer-matrix extension (configs 1 and 4): symmetric and asymmetric."""
    rng = np.random.default_rng(7000 + n)
    for k in range(6 if n <= 12 else 2):
        hi = 1000 if k % 2 == 0 else 8
        m = rng.integers(1, hi, size=(n, n)).astype(np.int32)
        if k % 3 != 2:
            m = np.minimum(m, m.T)
        np.fill_diagonal(m, 0)
        cost, tour, st = tspgpu.search_solve(gpu_ctx, m)
        oc, ot = O.solve_block(m.astype(np.float64))
        assert cost == int(oc), (n, k, st)
        assert tour.tolist() == ot, (n, k, st)


def test_clustered_16(gpu_ctx):
    """Config-4 stand-in: 4 Gaussian clusters (pruning imbalance across prefixes)."""
    rng = np.random.default_rng(44)
    for seed in range(3):
        centers = rng.uniform(100, 900, size=(4, 2))
        xy = np.concatenate([centers[i] + rng.normal(0, 50, size=(4, 2)) for i in range(4)])
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(16)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        oc, ot = O.solve_block(d)
        assert (cost, tour.tolist()) == (oc, ot), st


def test_k2_matches_k1(gpu_ctx):
    """Both GPU paths, same inputs: identical bits and tours (n = 12..16)."""
    rng = np.random.default_rng(99)
    for n in (12, 14, 16):
        xy = rng.uniform(0, 1000, size=(4, n, 2))
        blocks = [[(b * n + i, xy[b, i, 0], xy[b, i, 1]) for i in range(n)] for b in range(4)]
        d = tspgpu.distance_matrix(blocks)
        c1, t1 = gpu_ctx.solve_blocks(d)
        for b in range(4):
            c2, t2, _ = tspgpu.search_solve(gpu_ctx, d[b])
            assert c2 == c1[b] and t2.tolist() == t1[b].tolist()


@pytest.mark.parametrize("budget", ["1", "64"])
def test_tiny_budget_splits_everything(gpu_ctx, budget, knobs):
    """Round kernel (2), budgets of 1 and 64 iterations: nearly every item is
    cut and re-queued many times; the answer must not change."""
    knobs.set("SEARCH_KERNEL", "2")
    knobs.set("SEARCH_BUDGET", budget)
    rng = np.random.default_rng(int(budget))
    for n in (9, 12):
        xy = rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        oc, ot = O.solve_block(d)
        assert (cost, tour.tolist()) == (oc, ot), st
        if n == 12 and budget == "1":
            assert st["rounds"] > 2, st


@pytest.mark.parametrize("mode", ["donate_always", "small_ring", "kernel1", "kernel2"])
def test_search_kernels_and_hand_off_stress(gpu_ctx, mode, knobs):
    """Persistent search with a donation at every chance (every busy lane
    splits its root level whenever it may), with a 64-item ring (donations
    mostly refused by the capacity check), and the two round kernels: same
    cost and tour as the oracle, tie-heavy and random instances."""
    env = {"donate_always": {"SEARCH_HUNGRY": "-1000000000", "SEARCH_MIN_SPLIT": "0"},
           "small_ring": {"SEARCH_RING_LOG2": "6", "SEARCH_HUNGRY": "-1000000000", "SEARCH_MIN_SPLIT": "0"},
           "kernel1": {"SEARCH_KERNEL": "1"}, "kernel2": {"SEARCH_KERNEL": "2"}}[mode]
    for k, v in env.items():
        knobs.set(k, v)
    knobs.set("SEARCH_WALL_S", "30")
    rng = np.random.default_rng(len(mode))
    for n in (5, 9, 12, 14):
        for kind in ("ties", "random"):
            if kind == "ties":
                xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)
            else:
                xy = rng.uniform(0, 1000, size=(n, 2))
            d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            oc, ot = O.solve_block(d)
            assert (cost, tour.tolist()) == (oc, ot), (mode, n, kind, st)


@pytest.mark.parametrize("mode", [("0", None, None), ("5", None, None), ("6", None, None), ("6", "8", "2"),
                                  ("5", "8", "1"), ("6", None, "2")])
def test_frontier_search_modes(gpu_ctx, mode, knobs):
    """Frontier search (expand_kernel level by level, then the prefixes with
    5/6 cities left folded by tail_kernel) against the DFS rounds ("0"):
    default seed depth, shallow seeds (depth 1-2: many expansion levels) and
    a 256-slot tail buffer (a flush every few expansions, many small steps).
    Same cost and tour as the oracle on tie-heavy, random and integer
    instances, n = 8..14."""
    tail, cap, depth = mode
    knobs.set("SEARCH_TAIL", tail)
    if cap is not None:
        knobs.set("SEARCH_TAIL_CAP_LOG2", cap)
    if depth is not None:
        knobs.set("SEARCH_DEPTH", depth)
    rng = np.random.default_rng(17 + int(tail) + (0 if cap is None else 7) + (0 if depth is None else 3))
    for n in (8, 9, 11, 13, 14):
        for kind in ("ties", "random", "int"):
            if kind == "ties":
                xy = rng.integers(0, 5, size=(n, 2)).astype(np.float64)
            else:
                xy = rng.uniform(0, 1000, size=(n, 2))
            d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
            if kind == "int":
                d = np.rint(d).astype(np.int32)
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            oc, ot = O.solve_block(d.astype(np.float64))
            assert (float(cost), tour.tolist()) == (oc, ot), (mode, n, kind, st)


def test_frontier_16_golden(gpu_ctx, knobs):
    """The reference's own 16-city instance through the frontier search with
    5- and 6-city register tails: golden cost bits and tour."""
    case = next(c for c in O.load_golden("seed0_blocks.json") if c["n"] == 16 and c["B"] == 1 and c["X"] == 1000)
    blk = _cities(case["cities"][0])
    d = tspgpu.distance_matrix([blk])[0]
    for tail in ("5", "6"):
        knobs.set("SEARCH_TAIL", tail)
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        assert cost == O.hexf(case["solutions"][0]["cost_hex"]), st
        assert [blk[t][0] for t in tour] == case["solutions"][0]["ids"], st


@pytest.mark.parametrize("mode", ["chain", "steps", "chain_overflow"])
def test_chained_small_search(gpu_ctx, mode, knobs):
    """Small single-shard searches run as chained frontier levels (one
    synchronisation); a level that overflows the ping-pong buffers falls back
    to the stepwise search.  All three give the reference's golden 16-city
    answer, and random / tie-heavy instances equal the oracle."""
    if mode == "steps":
        knobs.set("SEARCH_CHAIN", "0")
    if mode == "chain_overflow":
        knobs.set("SEARCH_CHAIN_CAP_LOG2", "8")
    case = next(c for c in O.load_golden("seed0_blocks.json") if c["n"] == 16 and c["B"] == 1 and c["X"] == 1000)
    blk = _cities(case["cities"][0])
    d = tspgpu.distance_matrix([blk])[0]
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    assert cost == O.hexf(case["solutions"][0]["cost_hex"]), st
    assert [blk[t][0] for t in tour] == case["solutions"][0]["ids"], st
    rng = np.random.default_rng(11)
    for n in (9, 12, 14, 17, 18):
        for kind in ("random", "lattice"):
            xy = rng.uniform(0, 1000, size=(n, 2)) if kind == "random" else rng.integers(0, 4, size=(n, 2)) * 1.0
            dd = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
            c2, t2, s2 = tspgpu.search_solve(gpu_ctx, dd)
            assert (c2, t2.tolist()) == O.solve_block(dd), (mode, n, kind, s2)


@pytest.mark.parametrize("n", [22, 28])
def test_chained_search_with_tree_bound_above_18(gpu_ctx, n, knobs):
    """With the tree bound the chained levels run up to 32 cities: the same
    cost and tour as the stepwise search.  A chain whose level buffers
    overflow reruns step by step from its starting state: after a 32-city
    search in the same context (its paths left in the pooled buffers, which
    an overflowing block's unwritten slots expose), forced overflows — with
    and without the tree bound — still give the same answer."""
    from bench import k2_instance

    d = np.asarray(k2_instance(n, 3))
    c0, t0, _ = tspgpu.search_solve(gpu_ctx, d)
    knobs.set("SEARCH_CHAIN", "0")
    c1, t1, _ = tspgpu.search_solve(gpu_ctx, d)
    knobs.clear("SEARCH_CHAIN")
    assert c0 == c1 and t0.tolist() == t1.tolist()
    tspgpu.search_solve(gpu_ctx, np.asarray(k2_instance(32, 35)))
    knobs.set("SEARCH_CHAIN_CAP_LOG2", "10")
    c2, t2, _ = tspgpu.search_solve(gpu_ctx, d)
    assert c2 == c0 and t2.tolist() == t0.tolist()
    if n == 22:  # (without the tree bound the 28-city search takes seconds)
        knobs.set("SEARCH_MST", "0")
        c3, t3, _ = tspgpu.search_solve(gpu_ctx, d)
        assert c3 == c0 and t3.tolist() == t0.tolist()


@pytest.mark.parametrize("nshards", [2, 3, 5])
def test_sharded_on_one_gpu(gpu_ctx, nshards):
    """The multi-GPU decomposition, run shard by shard on one device: min of
    the shards' incumbents + union of their optimal records -> same answer."""
    rng = np.random.default_rng(nshards)
    n = 13
    xy = rng.integers(0, 5, size=(n, 2)).astype(np.float64)
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
    shards = [tspgpu.Search(gpu_ctx, d, shard=s, nshards=nshards) for s in range(nshards)]
    ub, _ = tspgpu.heuristic_tour(d)
    for S in shards:
        S.set_bound(ub)
        S.run_all()
    opt = min(S.counters()[0] for S in shards)
    recs = [r for S in shards for r in S.records(opt)]
    cost = tspgpu.bits_cost(opt, tspgpu.F64)
    tour = tspgpu.select_tour(d, recs, cost)
    oc, ot = O.solve_block(d)
    assert cost == oc and tour.tolist() == ot
    for S in shards:
        S.close()


def test_solve_sharded_single_process(gpu_ctx, knobs):
    """search_dist's driver with one rank (exchanges are no-ops): the shard as
    one device chain and the winner from the device tie key (one phase, no
    record read), also on tie-heavy lattices; step by step (chain off) with an
    exchange every step or every 4 steps."""
    rng = np.random.default_rng(5)
    for kind in ("random", "lattice", "lattice"):
        xy = rng.uniform(0, 1000, size=(15, 2)) if kind == "random" else rng.integers(0, 4, size=(15, 2)) * 1.0
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(15)])
        oc, ot = O.solve_block(d)
        cost, tour, st = search_dist.solve_sharded(gpu_ctx, d)
        assert cost == oc and tour.tolist() == ot, st
        assert st["chained"] == 1 and st["exchanges"] == 1, st
        assert st["phases"] == 1 and st["tie"] == 1 and st["record_gather"] == 0, st
    knobs.set("SEARCH_CHAIN", "0")
    cost, tour, st = search_dist.solve_sharded(gpu_ctx, d, exchange_every=1)
    assert cost == oc and tour.tolist() == ot, st
    assert st["chained"] == 0 and st["exchanges"] == st["rounds"] >= 1 and st["tie"] == 1
    # 4 steps per exchange: same answer, fewer exchanges
    cost, tour, st4 = search_dist.solve_sharded(gpu_ctx, d)
    assert cost == oc and tour.tolist() == ot, st4
    assert st4["exchange_every"] == 4 and 1 <= st4["exchanges"] <= st4["rounds"] // 4 + 1


@pytest.mark.parametrize("n", [22, 26])
def test_solve_sharded_two_word_keys(gpu_ctx, n):
    """n - 1 > 20 inner cities: the tie key spans two words (w0, then w1 among
    the holders of the least w0); the sharded driver's answer equals the
    one-GPU search's."""
    from bench import k2_instance

    d = np.asarray(k2_instance(n, 7))
    c0, t0, _ = tspgpu.search_solve(gpu_ctx, d)
    cost, tour, st = search_dist.solve_sharded(gpu_ctx, d)
    assert cost == c0 and tour.tolist() == t0.tolist(), st
    assert st["tie"] == 1 and st["record_gather"] == 0 and st["chained"] == 1, st


def test_chain_tie_slot_abi(gpu_ctx):
    """tspgpu_search_chain + tspgpu_search_tie_slot on shards run one after
    another: the MIN of the shards' keys at the MIN of their incumbents is
    tsp()'s tour (tspgpu_tie_tour certifies it)."""
    rng = np.random.default_rng(3)
    xy = rng.integers(0, 4, size=(15, 2)).astype(np.float64)  # (15 cities: a frontier search, so chained)
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(15)])
    ub, _ = tspgpu.heuristic_tour(d)
    shards = [tspgpu.Search(gpu_ctx, d, shard=s, nshards=3) for s in range(3)]
    try:
        for S in shards:
            S.set_bound(ub)
            assert S.chain()
        opt = min(S.counters()[0] for S in shards)
        slots = [S.tie_slot(opt) for S in shards]
        assert not any(ovf for _, _, _, ovf in slots), slots
        w0 = min(w for f, w, _, _ in slots if f)
        rc, tour = tspgpu.tie_tour(d, w0, 0, tspgpu.bits_cost(opt, tspgpu.F64))
        oc, ot = O.solve_block(d)
        assert rc == 0 and tspgpu.bits_cost(opt, tspgpu.F64) == oc and tour.tolist() == ot
        # the slot of a cost no shard recorded (every recorded tour costs at most the bound)
        assert all(not S.tie_slot(tspgpu.cost_bits(2 * ub + 1, tspgpu.F64))[0] for S in shards)
    finally:
        for S in shards:
            S.close()


def test_overflow_falls_back_to_second_phase(gpu_ctx, knobs):
    """All-equal distances: every tour is optimal.  7! = 5040 fit the record
    buffer; 9! = 362880 at n = 10 do not, so (device tie rule off) the search
    runs a second phase with the optimum as the bound and a buffer of the
    needed size.  With the device tie rule on, one phase answers it."""
    d = np.full((10, 10), 7, dtype=np.int32)
    np.fill_diagonal(d, 0)
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    oc, ot = O.solve_block(d.astype(np.float64))
    assert cost == int(oc) and tour.tolist() == ot and st["phases"] == 1 and st["tie"] == 1, st
    knobs.set("SEARCH_TIE", "0")
    d = np.full((8, 8), 7, dtype=np.int32)
    np.fill_diagonal(d, 0)
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)  # 7! = 5040 optimal tours: fits
    oc, ot = O.solve_block(d.astype(np.float64))
    assert cost == int(oc) and tour.tolist() == ot and st["optimal_tours"] == 5040
    d = np.full((10, 10), 7, dtype=np.int32)
    np.fill_diagonal(d, 0)
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    oc, ot = O.solve_block(d.astype(np.float64))
    assert cost == int(oc) and tour.tolist() == ot and st["phases"] == 2 and st["optimal_tours"] == 362880


def test_forced_second_phase_and_k1_fallback(gpu_ctx, knobs):
    """A tiny record buffer forces the second phase on an ordinary lattice
    instance; coincident cities (12! optimal tours) fall back to K1."""
    rng = np.random.default_rng(11)
    xy = rng.integers(0, 3, size=(11, 2)).astype(np.float64)
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(11)])
    knobs.set("SEARCH_RECORD_CAP", "2")
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)  # device tie rule: one phase
    oc, ot = O.solve_block(d)
    assert (cost, tour.tolist()) == (oc, ot) and st["phases"] == 1 and st["tie"] == 1, st
    knobs.set("SEARCH_TIE", "0")
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    knobs.clear("SEARCH_RECORD_CAP")
    assert (cost, tour.tolist()) == (oc, ot) and st["phases"] == 2, st
    d = np.zeros((13, 13))
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    oc, ot = O.solve_block(d)
    assert (cost, tour.tolist()) == (oc, ot) and st["fallback"] == 1, st


def test_coincident_cities_device_tie_rule(gpu_ctx):
    """12! optimal tours (13 coincident cities): the device tie rule answers in
    one phase, with neither a second search nor the K1-wide fallback."""
    d = np.zeros((13, 13))
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
    oc, ot = O.solve_block(d)
    assert (cost, tour.tolist()) == (oc, ot), st
    assert st["phases"] == 1 and st["fallback"] == 0 and st["tie"] == 1, st


@pytest.mark.parametrize("n", [9, 12, 14, 17])
def test_device_tie_rule_agrees_with_records(gpu_ctx, n, knobs):
    """Tie-heavy lattices and uniform cities.  Default: the records decide and
    the device answer, when certified cheaply, must agree (tie_checked != -1).
    With a 2-record buffer (as in a tie storm) the device tie rule decides in
    one phase (certified with the prefix DP) and gives the same tour — tsp()'s
    (oracle) up to 16 cities, the records' rule at 17."""
    rng = np.random.default_rng(77 + n)
    used = overflowed = 0
    for k in range(6):
        if k % 3 == 2:
            xy = rng.uniform(0, 1000, size=(n, 2))
        else:
            xy = rng.integers(0, 3 + k, size=(n, 2)).astype(np.float64)
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
        assert st["tie_checked"] != -1, st
        if n <= 16:
            oc, ot = O.solve_block(d)
            assert (cost, tour.tolist()) == (oc, ot), (k, st)
        knobs.set("SEARCH_RECORD_CAP", "2")
        c2, t2, s2 = tspgpu.search_solve(gpu_ctx, d)
        knobs.clear("SEARCH_RECORD_CAP")
        assert (c2, t2.tolist()) == (cost, tour.tolist()), (k, s2)
        if s2["tie"]:
            assert s2["phases"] == 1 and s2["fallback"] == 0, s2
        if s2["records"] > 2:  # the buffer overflowed: the device rule's case
            overflowed += 1
            used += s2["tie"]
    assert overflowed >= 1 and used >= overflowed - 1, (used, overflowed)


@pytest.mark.parametrize("n", [22, 26])
def test_device_tie_rule_two_word_keys(gpu_ctx, n, knobs):
    """Above 21 cities the key takes two words (a sub-slot per first word): the
    device answer equals the records' rule on symmetric instances (two optimal
    orientations at least), uniform and on a 40 x 40 lattice; a two-record
    buffer makes the device rule decide."""
    rng = np.random.default_rng(5 * n)
    for k in range(3):
        xy = rng.uniform(0, 1000, size=(n, 2)) if k == 0 else rng.integers(0, 40, size=(n, 2)).astype(np.float64)
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        knobs.clear("SEARCH_TIE")
        c1, t1, s1 = tspgpu.search_solve(gpu_ctx, d)
        knobs.set("SEARCH_RECORD_CAP", "1")
        c2, t2, s2 = tspgpu.search_solve(gpu_ctx, d)
        knobs.clear("SEARCH_RECORD_CAP")
        knobs.set("SEARCH_TIE", "0")
        c0, t0, s0 = tspgpu.search_solve(gpu_ctx, d)
        assert c1 == c0 and t1.tolist() == t0.tolist() and s1["tie_checked"] != -1, (k, s1, s0)
        assert c2 == c0 and t2.tolist() == t0.tolist(), (k, s2)


@pytest.mark.parametrize("n", [3, 4, 6, 8, 10, 11])
def test_exhaustive_enumeration_against_oracle(gpu_ctx, n):
    """No bound at all: every tour folded; same cost bits and tour as tsp()."""
    rng = np.random.default_rng(9000 + n)
    for lattice in (False, True):
        xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64) if lattice else rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
        oc, ot = O.solve_block(d)
        assert (cost, tour.tolist()) == (oc, ot), (n, lattice, st)
        # every complete tour is a node below the seed depth: at least (n-1)! of them
        import math
        assert st["nodes"] >= math.factorial(n - 1), (st["nodes"], n)


def test_exhaustive_14_golden(gpu_ctx):
    """BASELINE config 2: `./tsp 14 1 1000 1000` by exhaustive enumeration
    (13! = 6.2e9 tours) — the reference's golden cost and tour."""
    case = next(c for c in O.load_golden("seed0_blocks.json") if c["n"] == 14 and c["B"] == 1 and c["X"] == 1000)
    cities = _cities(case["cities"][0])
    d = tspgpu.distance_matrix([cities])[0]
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
    assert cost == O.hexf(case["solutions"][0]["cost_hex"]), st
    assert [cities[t][0] for t in tour] == case["solutions"][0]["ids"], st
    assert st["nodes"] > 6.0e9, st


def _enum_nodes(n):
    import math
    N = n - 1
    return sum(math.factorial(N) // math.factorial(N - l) for l in range(1, N + 1))


@pytest.mark.parametrize("n", [7, 9, 12, 13])
def test_enum_kernel_against_oracle_and_round_kernels(gpu_ctx, n, knobs):
    """enum.hip (7 <= n <= 16: a lane per depth-(n-7) prefix, 720 completions
    in registers) against tsp()'s oracle, on random and tie-heavy lattice
    cities; the round kernels with the bound off (knob ENUM_KERNEL=0) give
    the same answer; the node count is every partial path exactly."""
    rng = np.random.default_rng(9100 + n)
    for lattice in (False, True):
        xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64) if lattice else rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour, st = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
        oc, ot = O.solve_block(d)
        assert (cost, tour.tolist()) == (oc, ot), (n, lattice, st)
        assert st["nodes"] == _enum_nodes(n) and st["depth"] == n - 7, st
        if n <= 12:
            knobs.set("ENUM_KERNEL", "0")
            c2, t2, st2 = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
            knobs.clear("ENUM_KERNEL")
            assert (c2, t2.tolist()) == (oc, ot), (n, lattice, st2)


@pytest.mark.parametrize("n", [8, 12])
def test_enum_kernel_integer_matrix(gpu_ctx, n):
    """Integer distances (config 1 extension) through the enumeration kernel:
    exact int32 folds, same optimum and tie-broken tour as the int64 oracle."""
    rng = np.random.default_rng(77 + n)
    for hi in (1000, 5):
        m = rng.integers(1, hi + 1, size=(n, n)).astype(np.int32)
        m = np.triu(m, 1)
        m = m + m.T
        cost, tour, st = tspgpu.search_solve(gpu_ctx, m, exhaustive=True)
        oc, ot = O.solve_block(m.astype(np.int64))
        assert (cost, tour.tolist()) == (int(oc), ot), (n, hi, st)


def test_enum_kernel_record_overflow_second_phase(gpu_ctx, knobs):
    """Thousands of tied optima on a 3x3 lattice (n=10) with a 2-record
    buffer: the device tie rule answers in one phase; without it the
    enumeration runs a second phase with the optimum as the bound.  Both
    return tsp()'s tour."""
    xy = [(x, y) for x in range(3) for y in range(3)] + [(1.0, 0.5)]
    d = O.distance_matrix([(i, float(x), float(y)) for i, (x, y) in enumerate(xy)])
    oc, ot = O.solve_block(d)
    knobs.set("SEARCH_RECORD_CAP", "2")
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
    assert (cost, tour.tolist()) == (oc, ot) and st["phases"] == 1 and st["tie"] == 1, st
    knobs.set("SEARCH_TIE", "0")
    cost, tour, st = tspgpu.search_solve(gpu_ctx, d, exhaustive=True)
    assert (cost, tour.tolist()) == (oc, ot) and st["phases"] == 2, st


@pytest.mark.parametrize("kind", ["random", "clustered", "ties"])
def test_lagrangian_two_edge_bound_keeps_the_answer(gpu_ctx, kind, knobs):
    """The Lagrangian city weights only change which nodes are pruned: with
    and without them (knob SEARCH_LAGRANGE) the search returns the DP's cost
    and tour (K1-wide) on random and clustered instances of 17-21 cities and
    tie-heavy ones of 13-17."""
    rng = np.random.default_rng({"random": 1, "clustered": 2, "ties": 3}[kind])
    for n in ((13, 15, 17) if kind == "ties" else (17, 19, 21)):
        if kind == "random":
            xy = rng.uniform(0, 1000, size=(n, 2))
        elif kind == "clustered":
            c = rng.uniform(100, 900, size=(3, 2))
            xy = c[np.arange(n) % 3] + rng.normal(0, 40, size=(n, 2))
        else:
            xy = rng.integers(0, 6, size=(n, 2)).astype(np.float64)
        d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
        wc, wt, _ = gpu_ctx.solve_instance(d)
        for lag in ("1", "0"):
            knobs.set("SEARCH_LAGRANGE", lag)
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            assert cost == wc and tour.tolist() == wt.tolist(), (kind, n, lag, st)


@pytest.mark.parametrize("kind", ["random", "clustered", "ties", "integer"])
def test_tree_bound_keeps_the_answer(gpu_ctx, kind, knobs):
    """The Held-Karp tree bound (knob SEARCH_MST, on at paths with >= 12
    cities left by default, SEARCH_MST_MINREM=0: at every level) only
    changes which paths are pruned: off, default and everywhere, the search
    returns the DP's cost and tie-broken tour (K1-wide) on random, clustered,
    tie-heavy and integer (i32 search) instances of 13-25 cities."""
    rng = np.random.default_rng({"random": 11, "clustered": 12, "ties": 13, "integer": 14}[kind])
    for n in ((13, 16, 19) if kind in ("ties", "integer") else (18, 22, 25)):
        if kind == "clustered":
            c = rng.uniform(100, 900, size=(3, 2))
            xy = c[np.arange(n) % 3] + rng.normal(0, 40, size=(n, 2))
        elif kind == "ties":
            xy = rng.integers(0, 6, size=(n, 2)).astype(np.float64)
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        d = tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]
        if kind == "integer":
            d = np.rint(d).astype(np.int32)
        wc, wt, _ = gpu_ctx.solve_instance(np.asarray(d, dtype=np.float64))
        for mst, minrem in (("0", None), ("1", None), ("1", "0")):
            if mst == "0" and n >= 25:
                # (bound off at 25 clustered cities: 7e13 nodes, ~160 s of one
                # GPU — the answer is pinned by K1-wide with the bound on and at
                # 18 / 22 cities with it off; tools/k2_mst0_probe.py times it)
                continue
            knobs.set("SEARCH_MST", mst)
            if minrem is None:
                knobs.clear("SEARCH_MST_MINREM")
            else:
                knobs.set("SEARCH_MST_MINREM", minrem)
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            assert cost == wc and tour.tolist() == wt.tolist(), (kind, n, mst, minrem, st)


def test_tree_bound_on_the_hard_32_city_seeds(gpu_ctx, knobs):
    """bench.k2_instance(32, s) for the seeds whose two-edge bound left a
    heavy tail (35: 0.5 s without the tree bound; 14 and 20: 11-14 s): with
    the tree bound each is solved in well under a second, the same answer at
    every gating level, and seed 35 also equals the search without it."""
    from bench import k2_instance

    for seed in (35, 14, 20):
        d = k2_instance(32, seed)
        got = []
        for minrem in ("12", "0"):
            knobs.set("SEARCH_MST_MINREM", minrem)
            cost, tour, st = tspgpu.search_solve(gpu_ctx, d)
            assert st["kernel_ms"] < 500, st
            got.append((cost, tour.tolist()))
        assert got[0] == got[1], seed
        if seed == 35:
            knobs.set("SEARCH_MST", "0")
            cost, tour, _ = tspgpu.search_solve(gpu_ctx, d)
            knobs.clear("SEARCH_MST")
            assert (cost, tour.tolist()) == got[0]


@pytest.mark.parametrize("n,cap", [(16, 8), (22, 10)])
def test_chain_overflow_reads_no_unwritten_slot(knobs, n, cap):
    """A chained level that overflows leaves output slots it reserved but never
    wrote.  On a FRESH context whose level and tail buffers are filled with
    0xFF bytes (knob SEARCH_CHAIN_POISON: paths of length 255, cities 255 —
    out of range of every LDS table), a forced overflow (tiny level buffers)
    must still return the stepwise search's answer: the chained kernels after
    the overflow read no slot (they return at once) and the rerun starts from
    the chain's starting state."""
    from bench import Shard, k2_instance

    d = Shard(16, 1, 0, 1).distances()[0] if n == 16 else np.asarray(k2_instance(n, 3))
    ctx = tspgpu.Context(device=0)
    try:
        knobs.set("SEARCH_CHAIN_POISON", 1)
        knobs.set("SEARCH_CHAIN_CAP_LOG2", cap)
        c1, t1, s1 = tspgpu.search_solve(ctx, d)
        knobs.clear()
        knobs.set("SEARCH_CHAIN", 0)
        c0, t0, _ = tspgpu.search_solve(ctx, d)
    finally:
        ctx.close()
    assert c1 == c0 and t1.tolist() == t0.tolist(), s1
    if n == 16:
        assert c1 == 3871.1947567096445 and t1.tolist() == [0, 14, 2, 13, 10, 12, 6, 4, 9, 11, 3, 5, 15, 8, 1, 7, 0]


@pytest.mark.parametrize("n,seed", [(16, 0), (20, 4), (24, 5), (32, 35), (32, 14)])
def test_device_bound_and_record_certificate(gpu_ctx, knobs, n, seed):
    """Round 6: the create launch's device bound up to 32 cities
    (tspgpu_search_create_ex TSPGPU_SEARCH_DEVICE_BOUND, solve_sharded's
    default) and the certificate from the optimal records
    (tspgpu_tie_tour_records) give exactly the answer of the host-bound search
    and of the native solve with and without the device bound extended."""
    from bench import Shard, k2_instance

    d = Shard(16, 1, 0, 1).distances()[0] if n == 16 else np.asarray(k2_instance(n, seed))
    want = tspgpu.search_solve(gpu_ctx, d)
    knobs.set("SEARCH_DEVICE_BOUND_MAXN", "33")
    native_dev = tspgpu.search_solve(gpu_ctx, d)
    knobs.clear("SEARCH_DEVICE_BOUND_MAXN")
    dev = search_dist.solve_sharded(gpu_ctx, d, bound="device")
    host = search_dist.solve_sharded(gpu_ctx, d, bound="host")
    for cost, tour, st in (native_dev, dev, host):
        assert cost == want[0] and tour.tolist() == want[1].tolist(), (n, seed, st)
    assert dev[2]["bound"] == "device" and dev[2]["tie"] == 1 and dev[2]["record_gather"] == 0
    # the record certificate agrees with the GPU prefix-DP certificate
    S = tspgpu.Search(gpu_ctx, d, device_bound=True)
    try:
        assert S.chain()
        inc, _, _ = S.counters()
        found, w0, w1, ovf = S.tie_slot(inc)
        assert found and not ovf
        recs = S.records(inc)
        rc_r, t_r = tspgpu.tie_tour_records(gpu_ctx, d, w0, w1 if n - 1 > 20 else 0, want[0], recs)
        rc_g, t_g = tspgpu.tie_tour_gpu(gpu_ctx, d, w0, w1 if n - 1 > 20 else 0, want[0])
        assert rc_r == rc_g == 0 and t_r.tolist() == t_g.tolist() == want[1].tolist()
    finally:
        S.close()
