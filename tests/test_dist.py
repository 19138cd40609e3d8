"""The N>1 bench path on CPU: two gloo ranks run bench.py's own shard
assignment and timed-region plumbing (barrier, K steps, max over ranks) with
the CPU oracle standing in for the device step.  The product's GPU step is
exercised by the -m gpu tests; here we check the multi-rank orchestration."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, per_rank, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tsp-mpi-reduction_amd")]
    import bench
    import oracle_py as O

    group = bench.Group(world)
    lo, hi = bench.shard_bounds(rank, world, per_rank)
    shard = bench.Shard(n, per_rank * world, lo, hi)
    d = shard.distances()
    costs = []

    def step():
        costs.clear()
        for b in range(shard.B):
            costs.append(O.solve_block(d[b])[0])

    wall_max, wall = bench.timed_steps(step, lambda: None, group, warmup=1, steps=2)
    total = group.allsum(sum(costs))
    out.put((rank, lo, hi, [shard.block(b)[0][0] for b in range(shard.B)], wall_max, wall, total))
    group.dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_timing():
    import torch.multiprocessing as mp

    world, n, per_rank = 2, 8, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # contiguous, disjoint shards covering the global instance ./tsp n 12 1000 1000
    assert [(r[1], r[2]) for r in res] == [(0, 6), (6, 12)]
    first_ids = [i for r in res for i in r[3]]
    assert first_ids == [b * n for b in range(world * per_rank)]
    # the reported time is the max over ranks, identical on every rank
    assert res[0][4] == res[1][4] >= max(res[0][5], res[1][5])
    # the sum over both shards equals solving the whole instance
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import oracle_py as O

    whole = sum(O.solve_block(O.distance_matrix(b))[0] for b in O.generate(n, world * per_rank, 1000, 1000))
    assert abs(res[0][6] - whole) < 1e-6 * whole
