"""Every K1 variant the library can pick, checked block by block against the
CPU oracle at the sizes where it is the default — including the variant
switches that happen inside one call:

  * n = 16, B >= 2 x CUs: the restructured sub-cube kernel (variant 6,
    hk_sub.h) is the default; variant 5 (hk_tiled.h), variant 4 (ping-pong +
    parent words) and variant 2 are forced through the knob K1 (read when a
    context is created);
  * every variant-5/6 configuration compiled in (k1_cfg.h, knob TILED_CFG),
    f64 and i32;
  * tie-heavy blocks (integer lattice 0..3, 0..39) mixed with random ones;
  * one block solved alone (variant 2: fewer blocks than CUs) equals its row
    of the large batch (variant 5).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu

B_BIG = 520  # > 2 x 256 CUs: the large-batch defaults apply


def _blocks(n, B, seed):
    rng = np.random.default_rng(seed)
    blocks = []
    for b in range(B):
        if b % 3 == 0:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)  # heavy ties
        elif b % 3 == 1:
            xy = rng.integers(0, 40, size=(n, 2)).astype(np.float64)
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        blocks.append([(b * n + i, xy[i, 0], xy[i, 1]) for i in range(n)])
    return tspgpu.distance_matrix(blocks)


_ORACLE = {}


def _oracle_all(key, d):
    if key not in _ORACLE:
        with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
            _ORACLE[key] = list(ex.map(lambda b: O.solve_block(np.asarray(d[b], dtype=np.float64)),
                                       range(d.shape[0])))
    return _ORACLE[key]


def _ctx(variant=None, cfg=None):
    # (K1 knobs are read at context creation)
    try:
        for k, v in (("K1", variant), ("TILED_CFG", cfg)):
            if v is None:
                tspgpu.untune(k)
            else:
                tspgpu.tune(k, v)
        return tspgpu.Context(device=0)
    finally:
        tspgpu.untune("K1")
        tspgpu.untune("TILED_CFG")


def _check(ctx, d, ref, vb=8):
    if vb == 8:
        cost, tour = ctx.solve_blocks(d)
    else:
        cost, tour = ctx.solve_blocks_i32(d)
    n = d.shape[1]
    bad = [b for b in range(d.shape[0])
           if float(cost[b]) != ref[b][0] or tour[b][: tspgpu.tour_length(n)].tolist() != ref[b][1]]
    assert not bad, f"{len(bad)} blocks differ from the oracle, first {bad[:5]}"
    return ctx.last_variant()


@pytest.mark.parametrize("variant", [None, 6, 5, 4, 2])
def test_n16_large_batch_every_variant(variant):
    d = _blocks(16, B_BIG, 16)
    ref = _oracle_all(("f64", 16), d)
    ctx = _ctx(variant)
    try:
        used = _check(ctx, d, ref)
    finally:
        ctx.close()
    expect = 6 if variant is None else variant
    if variant == 5 and not any(v == 5 for v, *_ in _k1_cfgs()):
        expect = 4  # (no variant-5 forward kernel in a product build: the n = 16 fallback)
    assert used == expect


@pytest.mark.parametrize("n,vb,expect", [(13, 8, 6), (14, 8, 6), (15, 8, 6), (16, 8, 6), (12, 8, 2), (16, 4, 6),
                                         (15, 4, 2)])
def test_large_batch_default_per_size(n, vb, expect):
    """The large-batch default at each size (tspgpu.cpp: the sub-cube kernel
    at 13-16 cities f64 and 16 cities i32, the compact layer pass elsewhere),
    every block against the oracle."""
    d = _blocks(n, B_BIG, 40 + n)
    ref = _oracle_all(("f64", n, B_BIG, 40 + n), d)
    if vb == 4:
        d = np.rint(d).astype(np.int32)
        ref = _oracle_all(("i32", n, B_BIG, 40 + n), d.astype(np.float64))
    ctx = _ctx()
    try:
        assert _check(ctx, d, ref, vb) == expect
    finally:
        ctx.close()


def _k1_cfgs():
    """(variant, id, value bytes, n) of every configuration compiled into the
    library: the product rows of k1_cfg.h (sweep rows only in K1_SWEEP builds)."""
    import re

    path = os.path.join(os.path.dirname(tspgpu.PKG_DIR), "tsp-mpi-reduction_amd", "csrc", "k1_cfg.h")
    text = open(path).read()
    out = []
    for variant, macro in ((5, "TSPGPU_TILED_PRODUCT_CFGS"), (6, "TSPGPU_SUB_PRODUCT_CFGS")):
        body = text[text.index(f"#define {macro}(X)"):].split("\n\n", 1)[0]
        for m in re.finditer(r"X\((\d+), (\w+), (\d+), (\d+),", body):
            out.append((variant, int(m.group(1)), 8 if m.group(2) == "double" else 4, int(m.group(3)) + 1))
    return out


@pytest.mark.parametrize("variant,cfg,vb,n", _k1_cfgs())
def test_every_k1_configuration(variant, cfg, vb, n):
    d = _blocks(n, 300, 100 + n)
    ref = _oracle_all(("f64", n, 300), d)
    if vb == 4:
        d = np.rint(d).astype(np.int32)
        ref = _oracle_all(("i32", n, 300), d.astype(np.float64))
    ctx = _ctx(variant, cfg)
    try:
        assert _check(ctx, d, ref, vb) == variant
    finally:
        ctx.close()


def test_single_block_equals_its_row_of_the_big_batch(gpu_ctx):
    d = _blocks(16, B_BIG, 16)
    cost, tour = gpu_ctx.solve_blocks(d)
    assert gpu_ctx.last_variant() == 6
    for b in (0, 1, 2, 257, B_BIG - 1):
        c1, t1 = gpu_ctx.solve_blocks(d[b:b + 1])
        assert gpu_ctx.last_variant() == 2
        assert c1[0] == cost[b] and t1[0].tolist() == tour[b].tolist()


def test_back_to_back_launches_on_two_streams_share_the_workspace_safely(gpu_ctx):
    """Device entry points on one context but on two different streams, issued
    back to back without a host sync: the second launch waits for
    the first (they share the context's DP workspace), so both batches come out
    exactly as when solved one after the other."""
    da, db = _blocks(16, B_BIG, 31), _blocks(16, B_BIG, 32)
    ref_a, ref_b = gpu_ctx.solve_blocks(da), gpu_ctx.solve_blocks(db)
    s1, s2 = gpu_ctx.stream_create(), gpu_ctx.stream_create()
    bufs = []
    try:
        pa, pb = gpu_ctx.upload(da), gpu_ctx.upload(db)
        ca, cb = gpu_ctx.alloc(B_BIG * 8), gpu_ctx.alloc(B_BIG * 8)
        wa, wb = gpu_ctx.alloc(B_BIG * 17 * 4), gpu_ctx.alloc(B_BIG * 17 * 4)
        bufs = [pa, pb, ca, cb, wa, wb]
        for _ in range(3):
            gpu_ctx.solve_device(pa, 16, B_BIG, ca, wa, s1)
            gpu_ctx.solve_device(pb, 16, B_BIG, cb, wb, s2)
        gpu_ctx.synchronize(s1)
        gpu_ctx.synchronize(s2)
        assert np.array_equal(gpu_ctx.download(ca, (B_BIG,), np.float64), ref_a[0])
        assert np.array_equal(gpu_ctx.download(wa, (B_BIG, 17), np.int32), ref_a[1])
        assert np.array_equal(gpu_ctx.download(cb, (B_BIG,), np.float64), ref_b[0])
        assert np.array_equal(gpu_ctx.download(wb, (B_BIG, 17), np.int32), ref_b[1])
    finally:
        for p_ in bufs:
            gpu_ctx.free(p_)
        gpu_ctx.stream_destroy(s1)
        gpu_ctx.stream_destroy(s2)
