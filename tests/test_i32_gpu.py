"""K1 on integer distances (tspgpu_solve_blocks_i32): the same Held-Karp DP,
tie rule and tour layout on int32 matrices (TSPLIB-style rounded weights).

Parity: against the pinned CPU oracle (oracle/, tsp.cpp:405-509 restated) run
on the same matrix converted to double — every partial sum is an exact integer
below 2^31, so the f64 DP and the i32 DP take identical decisions — and against
the f64 GPU path.  Bit-exact on cost and tour.
"""
import errno

import numpy as np
import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu


def _int_blocks(rng, n, B):
    d = np.empty((B, n, n), dtype=np.int32)
    for b in range(B):
        if b % 3 == 0:
            m = rng.integers(0, 4, size=(n, n))          # heavy ties
        elif b % 3 == 1:
            m = rng.integers(0, 1_000_000, size=(n, n))   # asymmetric, wide range
        else:
            xy = rng.integers(0, 1000, size=(n, 2))       # rounded Euclidean (TSPLIB EUC_2D)
            m = np.rint(np.hypot(xy[:, None, 0] - xy[None, :, 0], xy[:, None, 1] - xy[None, :, 1]))
        d[b] = m
        np.fill_diagonal(d[b], 0)
    return d


@pytest.mark.parametrize("n", list(range(2, 21)))
def test_i32_against_oracle(gpu_ctx, n):
    rng = np.random.default_rng(5000 + n)
    B = 36 if n <= 13 else (9 if n <= 16 else 2)
    d = _int_blocks(rng, n, B)
    cost, tour = gpu_ctx.solve_blocks_i32(d)
    assert cost.dtype == np.int32
    c64, t64 = gpu_ctx.solve_blocks(d.astype(np.float64))
    L = tspgpu.tour_length(n)
    for b in range(B):
        oc, ot = O.solve_block(d[b].astype(np.float64))
        assert float(cost[b]) == oc, (n, b)
        assert tour[b][:L].tolist() == ot, (n, b)
        assert all(t == -1 for t in tour[b][L:])
    assert np.array_equal(cost.astype(np.float64), c64)
    assert np.array_equal(tour, t64)


def test_i32_full_size_properties(gpu_ctx):
    """n = 16, 2048 blocks: tours are permutations from/to 0, the integer fold of
    each tour equals its cost, and the result equals the f64 path's."""
    rng = np.random.default_rng(99)
    B, n = 2048, 16
    d = rng.integers(0, 100_000, size=(B, n, n)).astype(np.int32)
    cost, tour = gpu_ctx.solve_blocks_i32(d)
    c64, t64 = gpu_ctx.solve_blocks(d.astype(np.float64))
    assert np.array_equal(cost.astype(np.float64), c64) and np.array_equal(tour, t64)
    for b in range(0, B, 7):
        t = tour[b]
        assert t[0] == 0 and t[n] == 0 and sorted(t[:n].tolist()) == list(range(n))
        assert sum(int(d[b, t[i], t[i + 1]]) for i in range(n)) == int(cost[b])


def test_i32_validation_and_device_entry(gpu_ctx):
    with pytest.raises(tspgpu.TspGpuError) as e:
        gpu_ctx.solve_blocks_i32(np.full((1, 4, 4), -1, dtype=np.int32))
    assert e.value.code == -errno.EINVAL
    with pytest.raises(tspgpu.TspGpuError) as e:
        gpu_ctx.solve_blocks_i32(np.full((1, 4, 4), 600_000_000, dtype=np.int32))
    assert e.value.code == -errno.ERANGE
    c, _ = gpu_ctx.solve_blocks_i32(np.zeros((0, 5, 5), dtype=np.int32))
    assert c.shape == (0,)

    rng = np.random.default_rng(3)
    n, B = 15, 300
    d = rng.integers(0, 5000, size=(B, n, n)).astype(np.int32)
    ref_c, ref_t = gpu_ctx.solve_blocks_i32(d)
    dd = gpu_ctx.upload(d)
    dc = gpu_ctx.alloc(B * 4)
    dt = gpu_ctx.alloc(B * (n + 1) * 4)
    try:
        gpu_ctx.solve_device_i32(dd, n, B, dc, dt, gpu_ctx.stream)
        gpu_ctx.synchronize()
        assert np.array_equal(gpu_ctx.download(dc, (B,), np.int32), ref_c)
        got_t = gpu_ctx.download(dt, (B, n + 1), np.int32)
        assert np.array_equal(got_t[:, : n + 1], ref_t)
    finally:
        for p in (dd, dc, dt):
            gpu_ctx.free(p)
