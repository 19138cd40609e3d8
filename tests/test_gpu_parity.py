"""GPU parity: libtspgpu (gfx950 Held-Karp, called through the C ABI) against
the reference's own fixtures and the pinned CPU oracle.  Bit-exact on costs
(FP64 compared by value == bits) and tours (local indices / city ids).

Run on an MI355X:  python -m pytest tests -m gpu
"""
import numpy as np
import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu


def _solve_blocks_of_cities(ctx, blocks):
    d = tspgpu.distance_matrix(blocks)
    cost, tour = ctx.solve_blocks(d)
    return d, cost, tour


def _ids(blk, tour_row, n):
    L = tspgpu.tour_length(n)
    assert all(t == -1 for t in tour_row[L:])
    return [blk[t][0] for t in tour_row[:L]]


def test_seed0_fixtures(gpu_ctx):
    """Every block of the reference's own generated instances (n = 2..16)."""
    for case in O.load_golden("seed0_blocks.json"):
        blocks = [[(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in blk] for blk in case["cities"]]
        _, cost, tour = _solve_blocks_of_cities(gpu_ctx, blocks)
        for b, sol in enumerate(case["solutions"]):
            assert cost[b] == O.hexf(sol["cost_hex"]), (case["n"], case["B"], b)
            assert _ids(blocks[b], tour[b], case["n"]) == sol["ids"], (case["n"], case["B"], b)


@pytest.mark.parametrize("name", ["tie_blocks.json", "random_blocks.json"])
def test_file_fixtures(gpu_ctx, name):
    """Tie-heavy (collinear, lattice, coincident) and random instances."""
    data = O.load_golden(name)
    by_n = {}
    for inst in data:
        by_n.setdefault(len(inst["cities"]), []).append(inst)
    for n, insts in by_n.items():
        blocks = [[(c[0], O.hexf(c[1]), O.hexf(c[2])) for c in inst["cities"]] for inst in insts]
        _, cost, tour = _solve_blocks_of_cities(gpu_ctx, blocks)
        for b, inst in enumerate(insts):
            assert cost[b] == O.hexf(inst["solution"]["cost_hex"]), (name, n, b)
            assert _ids(blocks[b], tour[b], n) == inst["solution"]["ids"], (name, n, b)


@pytest.mark.parametrize("n", list(range(2, 21)))
def test_against_oracle_random(gpu_ctx, n):
    """Seeded random and integer-coordinate instances, every n incl. the n>16 extension."""
    rng = np.random.default_rng(1000 + n)
    B = 48 if n <= 13 else (12 if n <= 16 else 2)
    blocks = []
    for b in range(B):
        if b % 3 == 0:
            xy = rng.integers(0, 4, size=(n, 2)).astype(np.float64)  # heavy ties
        else:
            xy = rng.uniform(0, 1000, size=(n, 2))
        blocks.append([(b * n + i, xy[i, 0], xy[i, 1]) for i in range(n)])
    d, cost, tour = _solve_blocks_of_cities(gpu_ctx, blocks)
    for b in range(B):
        oc, ot = O.solve_block(d[b])
        assert cost[b] == oc, (n, b)
        assert tour[b][: tspgpu.tour_length(n)].tolist() == ot, (n, b)


def test_tour_cost_is_left_fold_and_permutation(gpu_ctx):
    """Full-size property (n=16, 1024 blocks): each tour is a permutation of the
    block starting/ending at 0, and its left-fold cost equals the returned cost
    bit for bit (the DP value is the left fold of its own argmin path)."""
    rng = np.random.default_rng(77)
    B, n = 1024, 16
    xy = rng.uniform(0, 1000, size=(B, n, 2))
    blocks = [[(b * n + i, xy[b, i, 0], xy[b, i, 1]) for i in range(n)] for b in range(B)]
    d, cost, tour = _solve_blocks_of_cities(gpu_ctx, blocks)
    for b in range(B):
        t = tour[b]
        assert t[0] == 0 and t[n] == 0 and sorted(t[:n].tolist()) == list(range(n))
        acc = 0.0
        for i in range(n):
            acc = acc + d[b, t[i], t[i + 1]]
        assert acc == cost[b]
    # spot-check optimality on a sample against the oracle
    for b in range(0, B, 97):
        assert O.solve_block(d[b])[0] == cost[b]


def test_deterministic_and_batch_independent(gpu_ctx):
    rng = np.random.default_rng(3)
    n = 15
    xy = rng.uniform(0, 1000, size=(600, n, 2))
    blocks = [[(i, p[0], p[1]) for i, p in enumerate(xy[b])] for b in range(600)]
    d = tspgpu.distance_matrix(blocks)
    c1, t1 = gpu_ctx.solve_blocks(d)
    c2, t2 = gpu_ctx.solve_blocks(d)
    c3, t3 = gpu_ctx.solve_blocks(d[123:124])
    assert np.array_equal(c1, c2) and np.array_equal(t1, t2)
    assert c3[0] == c1[123] and np.array_equal(t3[0], t1[123])


def test_validation_errors(gpu_ctx):
    import errno

    d = np.zeros((1, 4, 4))
    d[0, 1, 2] = np.inf
    with pytest.raises(tspgpu.TspGpuError) as e:
        gpu_ctx.solve_blocks(d)
    assert e.value.code == -errno.EINVAL
    d = np.full((1, 4, 4), 1e9)
    with pytest.raises(tspgpu.TspGpuError) as e:
        gpu_ctx.solve_blocks(d)
    assert e.value.code == -errno.ERANGE
    with pytest.raises(tspgpu.TspGpuError):
        gpu_ctx.solve_blocks(np.zeros((1, 1, 1)))
    strict = tspgpu.Context(device=0, strict=True)
    with pytest.raises(tspgpu.TspGpuError):
        strict.solve_blocks(np.zeros((1, 17, 17)))
    strict.close()
    c, t = gpu_ctx.solve_blocks(np.zeros((0, 5, 5)))
    assert c.shape == (0,)


def test_device_resident_entry_and_timer(gpu_ctx):
    """Device-pointer entry on the context's own stream (what bench.py times)."""
    rng = np.random.default_rng(9)
    n, B = 16, 256
    xy = rng.uniform(0, 1000, size=(B, n, 2))
    blocks = [[(i, p[0], p[1]) for i, p in enumerate(xy[b])] for b in range(B)]
    d = tspgpu.distance_matrix(blocks)
    ref_c, ref_t = gpu_ctx.solve_blocks(d)
    dd = gpu_ctx.upload(d)
    dc = gpu_ctx.alloc(B * 8)
    dt = gpu_ctx.alloc(B * (n + 1) * 4)
    try:
        gpu_ctx.timer_start()
        gpu_ctx.solve_device(dd, n, B, dc, dt, gpu_ctx.stream)
        ms = gpu_ctx.timer_stop()
        assert ms > 0
        assert np.array_equal(gpu_ctx.download(dc, (B,), np.float64), ref_c)
        got_t = gpu_ctx.download(dt, (B, n + 1), np.int32)
        assert np.array_equal(got_t, ref_t)
    finally:
        for p in (dd, dc, dt):
            gpu_ctx.free(p)


TORCH_INTEROP = r"""
import sys, numpy as np, torch
torch.cuda.init()                       # torch's HIP runtime first: libtspgpu binds to it
sys.path.insert(0, sys.argv[1])
import tspgpu
rng = np.random.default_rng(9)
n, B = 16, 64
xy = rng.uniform(0, 1000, size=(B, n, 2))
d = tspgpu.distance_matrix([[(i, p[0], p[1]) for i, p in enumerate(xy[b])] for b in range(B)])
ctx = tspgpu.Context(device=0)
ref_c, ref_t = ctx.solve_blocks(d)
dd = torch.from_numpy(d).cuda()
dc = torch.empty(B, dtype=torch.float64, device="cuda")
dt = torch.full((B, n + 1), -1, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
ctx.solve_device(dd.data_ptr(), n, B, dc.data_ptr(), dt.data_ptr(), s.cuda_stream)
s.synchronize()
assert np.array_equal(dc.cpu().numpy(), ref_c)
assert np.array_equal(dt.cpu().numpy(), ref_t)
print("OK")
"""


def test_torch_tensors_and_stream_interop():
    """torch-owned device tensors and a torch stream through the C ABI.  torch
    ships its own HIP runtime, so this runs in a fresh process that initialises
    torch first (libtspgpu then binds to the already-loaded runtime)."""
    import subprocess
    import sys

    pytest.importorskip("torch")
    p = subprocess.run([sys.executable, "-c", TORCH_INTEROP, tspgpu.PKG_DIR], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0 and "OK" in p.stdout, p.stderr[-2000:]


@pytest.mark.parametrize("variant", ["default", "2"])
@pytest.mark.parametrize("case", O.load_golden("k1_batches.json"), ids=lambda c: f"n{c['n']}")
def test_k1_batches_reference_goldens_default_kernel(gpu_ctx, case, variant, knobs):
    """The reference's own tsp() outputs for 522 blocks per n = 13..16 (tie-heavy
    lattices and uniform cities), solved in ONE batch: a batch of more than
    one block per CU runs the large-batch kernel — variant 6 (hk_sub_kernel,
    the default: the configuration ./tsp 16 65536 times) and variant 5
    and the layer-by-layer kernel (variant 2, knob K1=2) — both against the
    reference itself.  (Variant 5's forward kernels ship only in K1_SWEEP
    builds: test_k1_variants_gpu covers every configuration compiled in.)"""
    blocks = O.k1_batch_blocks(case)
    n = case["n"]
    ctx = gpu_ctx
    if variant != "default":
        knobs.set("K1", variant)
        ctx = tspgpu.Context(device=0)
    _, cost, tour = _solve_blocks_of_cities(ctx, blocks)
    assert ctx.last_variant() == (6 if variant == "default" else int(variant)), ctx.last_variant()
    if ctx is not gpu_ctx:
        ctx.close()
    bad = [b for b, ref in enumerate(case["blocks"])
           if cost[b] != O.hexf(ref["cost_hex"]) or _ids(blocks[b], tour[b], n) != ref["ids"]]
    assert not bad, f"n={n}: mismatching blocks {bad[:10]}"
