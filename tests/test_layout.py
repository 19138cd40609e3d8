"""CPU check of the K1 kernel's table layout and index arithmetic
(tsp-mpi-reduction_amd/csrc/heldkarp.hip: position-major layers,
G[S][k] at off(t) + pos(k in S) * C(N,t) + colexrank(S)), emulated step by step in Python:
colex ranks, layer offsets, the prefix/suffix destination-rank update and the
backtracking addresses.  Verifies that every table slot is written exactly
once, every read hits a written slot, no index leaves its layer, and the
emulated DP reproduces the oracle bit-exactly.  (The GPU itself is exercised
in test_gpu_parity.py.)
"""
import math

import numpy as np
import pytest

import oracle_py as O

INT_MAX = 2147483647.0


def layer_info(N):
    off, count, moff = {}, {}, {}
    o = m = 0
    for t in range(0, N + 2):
        count[t] = math.comb(N, t)
        moff[t] = m
        m += count[t]
        if t >= 1:
            off[t] = o
            o += count[t] * t
    masks = [x for t in range(N + 1) for x in range(1 << N) if bin(x).count("1") == t]
    return off, count, moff, masks, o


def C(a, b):
    return math.comb(a, b) if 0 <= b <= a else 0


def colex_rank(mask):
    r, j = 0, 0
    while mask:
        b = (mask & -mask).bit_length() - 1
        r += C(b, j + 1)
        j += 1
        mask &= mask - 1
    return r


def emulate(d):
    n = d.shape[0]
    N = n - 1
    off, count, moff, masks, total = layer_info(N)
    assert total == N << (N - 1)
    tab = np.full(total, np.nan)
    writes = np.zeros(total, dtype=np.int64)
    for i in range(N):
        tab[off[1] + i] = d[0, i + 1]  # rank i, position 0
        writes[off[1] + i] += 1
    for t in range(1, N):
        s = t + 1
        for r in range(count[t]):
            T = masks[moff[t] + r]
            assert bin(T).count("1") == t and colex_rank(T) == r
            row = [tab[off[t] + j * count[t] + r] for j in range(t)]
            assert not any(np.isnan(row))
            members = [k + 1 for k in range(N) if T >> k & 1]
            acc = [INT_MAX] * N
            for j, m in enumerate(members):
                for k in range(N):
                    acc[k] = min(acc[k], row[j] + d[m, k + 1])
            # descending k with suffix sums (heldkarp_impl.h scatter_row)
            q = s1 = s2 = 0
            for k in range(N - 1, -1, -1):
                inn = T >> k & 1
                p = t - q - inn
                c1, c2 = C(k, p + 1), C(k, p + 2)
                if not inn:
                    rank = r - s1 + c1 + s2
                    assert rank == colex_rank(T | (1 << k)) and rank < count[s]
                    a = off[s] + p * count[s] + rank
                    assert off[s] <= a < off[s] + count[s] * s
                    tab[a] = acc[k]
                    writes[a] += 1
                else:
                    s1 += c1
                    s2 += c2
                    q += 1
    assert (writes == 1).all()
    # closing + backtracking exactly as the kernel's wave does it
    full = (1 << N) - 1
    cands = [tab[off[N] + (m - 1) * count[N] + 0] + d[m, 0] for m in range(1, N + 1)]
    best = min(min(cands), INT_MAX)
    bestM = next(m for m in range(1, N + 1) if cands[m - 1] == best)
    tour = [0] * (n + 1)
    tour[n - 1] = bestM
    S, k, pos = full, bestM, n - 2
    while bin(S).count("1") >= 2:
        T = S & ~(1 << (k - 1))
        tt, ss = bin(T).count("1"), bin(T).count("1") + 1
        target = tab[off[ss] + bin(S & ((1 << (k - 1)) - 1)).count("1") * count[ss] + colex_rank(S)]
        pick = None
        for m in range(1, N + 1):
            if T >> (m - 1) & 1:
                c = tab[off[tt] + bin(T & ((1 << (m - 1)) - 1)).count("1") * count[tt] + colex_rank(T)] + d[m, k]
                if c == target:
                    pick = m
                    break
        assert pick is not None
        tour[pos] = pick
        pos -= 1
        S, k = T, pick
    assert pos == 0
    return best, tour


@pytest.mark.parametrize("n", [3, 4, 5, 6, 7, 8, 9])
def test_emulated_kernel_matches_oracle(n):
    rng = np.random.default_rng(n)
    for trial in range(6):
        if trial % 2:
            xy = rng.integers(0, 3, size=(n, 2)).astype(float)
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])
        cost, tour = emulate(d)
        oc, ot = O.solve_block(d)
        assert cost == oc and tour == ot


@pytest.mark.parametrize("N", list(range(2, 20)))
def test_layer_sizes_fit_kernel_constants(N):
    # heldkarp.h: LayerInfo arrays hold 24 entries, binomials C(a<=20, b<=23)
    off, count, moff, masks, total = layer_info(N)
    assert N + 1 < 24
    assert total == N << (N - 1)
    assert max(count.values()) < 2 ** 31
    assert len(masks) == 1 << N
