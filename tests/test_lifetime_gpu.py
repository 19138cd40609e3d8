"""Handle lifetimes of the C ABI (include/tspgpu.h "Destroy order is free").

Round 4's segfault (gpurun_out/r04_k2dist_tests.log): a failing test left
three tspgpu_search handles alive; the context fixture then called
tspgpu_ctx_destroy, which called the search pool's free function with the
pool pointer a live search had taken (null) — free_buffers(*nullptr) — and
any search destroyed afterwards would have dereferenced the freed context
(s->ctx->device, ->stream, ->mu, the pool).  Now every search holds a
reference on its context; destroying the context first only marks it closing.

  * bin/check_lifetime_asan: the library's host code under AddressSanitizer
    (built by the Makefile, -Xarch_host -fsanitize=address), context destroyed
    before live searches, the leak order, and the chain readback after a
    caller-written incumbent word;
  * the same order through the Python binding (no WeakSet bookkeeping left).
"""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu

ASAN_BIN = os.path.join(os.path.dirname(tspgpu.TSP_BIN), "check_lifetime_asan")


def test_lifetime_under_host_asan():
    assert os.path.exists(ASAN_BIN), "build it: make -C tsp-mpi-reduction_amd"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0")
    p = subprocess.run([ASAN_BIN], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "check_lifetime: ok" in p.stdout and "ERROR: AddressSanitizer" not in p.stderr


def test_context_closed_before_searches():
    rng = np.random.default_rng(3)
    xy = rng.uniform(0, 1000, size=(15, 2))
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(15)])
    oc, ot = O.solve_block(d)
    ctx = tspgpu.Context(device=0)
    ub, _ = tspgpu.heuristic_tour(d)
    shards = [tspgpu.Search(ctx, d, shard=s, nshards=3) for s in range(3)]
    for S in shards:
        S.set_bound(ub)
    ctx.close()  # before the searches: they keep the context alive
    best = None
    for S in shards:
        if not S.chain():
            S.run_all()
        inc = S.counters()[0]
        best = inc if best is None else min(best, inc)
    assert tspgpu.bits_cost(best, tspgpu.F64) == oc
    for S in reversed(shards):
        S.close()  # the last one releases the context
