"""search_dist.solve_sharded — the multi-GPU K2 driver — with world_size 2 and
3 over gloo.

CPU part: the driver's collective logic (incumbent all-reduce MIN between
rounds, "anyone busy" termination, all-gather of the optimal records, the
second phase when a rank lost records, the DP tie rule) runs with a
brute-force stand-in for the device search, so it is checked without a GPU.
GPU part (-m gpu): the real libtspgpu search, two ranks sharing device 0.
"""
import itertools
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class FakeSearch:
    """CPU stand-in for tspgpu.Search with the same shard semantics (depth-1
    prefix p = first city - 1 belongs to shard p mod S), one tour per round,
    records of every tour at cost <= incumbent, optional record capacity."""

    cap = 1 << 30

    def __init__(self, ctx, dist, shard=0, nshards=1, depth=0):
        import tspgpu

        self.dist, self.dtype = tspgpu._search_dist(dist)
        self.n = self.dist.shape[0]
        self.depth, self.items = 1, self.n - 1
        self.local_items = len(range(shard, self.items, nshards))
        self.tours = [p for p in itertools.permutations(range(1, self.n)) if (p[0] - 1) % nshards == shard]
        self.inc = None
        self.nodes = 0
        self.recs = []
        self.claimed = 0
        self.rounds = 0

    def _fold(self, t):
        c = self.dist.dtype.type(0)
        prev = 0
        for x in t:
            c = c + self.dist[prev, x]
            prev = x
        return c + self.dist[prev, 0]

    def set_bound(self, bound):
        import tspgpu

        self.inc = tspgpu.cost_bits(bound, self.dtype)

    def start(self):
        self.queue = list(self.tours)

    def step(self):
        import tspgpu

        self.rounds += 1
        if self.queue:
            t = self.queue.pop(0)
            self.nodes += 1
            bits = tspgpu.cost_bits(self._fold(t), self.dtype)
            if bits <= self.inc:
                self.inc = bits
                self.claimed += 1
                if len(self.recs) < self.cap:
                    self.recs.append((bits, t))
        return len(self.queue)

    def run_all(self):
        self.start()
        while self.step():
            pass

    def counters(self):
        return self.inc, self.nodes, self.claimed

    def reset_records(self, capacity=0):
        self.recs, self.claimed = [], 0
        self.cap = max(self.cap, capacity)

    def records(self, bits):
        import errno

        import tspgpu

        if self.claimed > self.cap:
            raise tspgpu.TspGpuError(-errno.EOVERFLOW, "fake")
        out = []
        for b, t in self.recs:
            if b == bits:
                r = tspgpu.TourRecord()
                r.cost = b
                for i, x in enumerate(t):
                    r.city[i] = x
                out.append(r)
        return out

    def timing(self):
        return 0.0, self.rounds

    def close(self):
        pass


def _cpu_worker(rank, world, port, dist, cap, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tsp-mpi-reduction_amd")]
    import torch.distributed as tdist

    import search_dist
    import tspgpu

    FakeSearch.cap = cap
    search_dist.tspgpu.Search = FakeSearch
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    cost, tour, st = search_dist.solve_sharded(None, dist)
    out.put((rank, cost, tour.tolist(), st["optimal_tours"], st["phases"], st["nodes"]))
    tdist.destroy_process_group()


def _run(worker, world, *args):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _lattice(n, seed):
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import oracle_py as O

    rng = np.random.default_rng(seed)
    xy = rng.integers(0, 3, size=(n, 2)).astype(np.float64)
    return O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(n)])


@pytest.mark.parametrize("world,cap", [(2, 1 << 30), (3, 1 << 30), (2, 1)])
def test_driver_collectives_cpu(world, cap):
    """Same cost and tour as the oracle on every rank; cap=1 forces the
    records-lost path (second phase on every rank)."""
    import oracle_py as O

    d = _lattice(7, 5 + world)
    res = _run(_cpu_worker, world, d, cap)
    oc, ot = O.solve_block(d)
    for rank, cost, tour, n_opt, phases, nodes in res:
        assert cost == oc and tour == ot
        assert n_opt >= 1 and nodes >= 720
        assert phases == (2 if cap == 1 else 1)


def _gpu_worker(rank, world, port, dist, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tsp-mpi-reduction_amd")]
    import torch.distributed as tdist

    import search_dist
    import tspgpu

    tdist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = tspgpu.Context(device=0)
    cost, tour, st = search_dist.solve_sharded(ctx, dist)
    ctx.close()
    out.put((rank, cost, tour.tolist(), st["rank_nodes"], st["nodes"], st["exchanges"]))
    tdist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_share_one_gpu():
    """The real sharded search: two processes, one GPU, gloo exchange."""
    import oracle_py as O

    rng = np.random.default_rng(21)
    xy = rng.uniform(0, 1000, size=(14, 2))
    d = O.distance_matrix([(i, xy[i, 0], xy[i, 1]) for i in range(14)])
    res = _run(_gpu_worker, 2, d)
    oc, ot = O.solve_block(d)
    assert all(cost == oc and tour == ot for _, cost, tour, *_ in res)
    assert res[0][4] == res[0][3] + res[1][3]  # total nodes = sum over ranks
    assert res[0][5] == res[1][5] >= 1          # same number of exchanges
