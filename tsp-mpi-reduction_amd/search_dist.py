"""Multi-GPU driver of K2 (one process per GPU, torch.distributed).

One instance is split over the ranks of a process group: rank r searches the
seed prefixes p with p mod W == r (libtspgpu's static shard); inside its GPU
the work runs in rounds (a device queue hands items to lanes, items that
exceed their budget are split and re-queued).  Between rounds the ranks
all-reduce(MIN) the 64-bit incumbent word (IEEE bits of the
f64 cost or the integer cost; both order like signed int64 for the
non-negative costs the ABI accepts), so every GPU prunes with the best tour
found anywhere.  At the end: all-reduce(MIN) of the incumbent = the optimum,
all-gather of each rank's records at that cost (the optimal set O), and every
rank applies the DP's tie rule (tspgpu_select_tour) to O — the same answer as
tsp() / K1 on one GPU.

With the "nccl" backend (RCCL on ROCm) the exchange is a device all-reduce
over xGMI; "gloo" runs the same logic over host tensors (CPU tests, or several
ranks sharing one GPU).  This replaces the reference's hand-rolled binary
MPI_Send/MPI_Recv tree (tsp.cpp:52-134) for the one step of the search that
needs a reduction: picking the global best tour.
"""
from __future__ import annotations

import errno
import os
import threading
import time

import numpy as np

import tspgpu


def _word_tensor(value: int, device):
    import torch

    return torch.tensor([value], dtype=torch.int64, device=device)


def solve_sharded(ctx, dist, group=None, depth: int = 0, device=None, exchange_every: int | None = None):
    """Search one instance over the ranks of `group` (None: the default group,
    or a single process when torch.distributed is not initialised).

    Every rank runs `exchange_every` steps of its own shard (fewer once it runs
    out of work), then all ranks exchange once: ONE all-reduce(MIN) of the pair
    (incumbent word, -busy).  The count is the same on every rank, so the
    collectives always pair up; a rank without work only joins the exchanges.
    Default: TSPGPU_EXCHANGE_EVERY or 4.

    Returns (cost, tour (n+1,), stats dict); identical on every rank."""
    import torch
    import torch.distributed as tdist

    dist_on = tdist.is_available() and tdist.is_initialized()
    rank = tdist.get_rank(group) if dist_on else 0
    world = tdist.get_world_size(group) if dist_on else 1
    backend = tdist.get_backend(group) if dist_on else "none"
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    # an nccl group runs every collective, even with one rank (a one-rank RCCL
    # communicator: the device all-reduce path exercised on a one-GPU box)
    collective = world > 1 or backend == "nccl"

    def allmin(word: int) -> int:
        if not collective:
            return word
        t = _word_tensor(word, device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN, group=group)
        return int(t.item())

    def allmin2(a: int, b: int):
        if not collective:
            return a, b
        import torch

        t = torch.tensor([a, b], dtype=torch.int64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN, group=group)
        v = t.tolist()
        return int(v[0]), int(v[1])

    if exchange_every is None:
        exchange_every = int(os.environ.get("TSPGPU_EXCHANGE_EVERY", "4"))
    exchange_every = max(1, int(exchange_every))

    # the multi-start tour (host, split over the ranks: start cities r, r+W,
    # ...) on a thread while the search is created (ctypes releases the GIL)
    heur = {}

    def _heuristic():
        heur["v"] = tspgpu.heuristic_tour(dist, first=rank, step=world) if world > 1 else \
            tspgpu.heuristic_tour(dist)

    th = threading.Thread(target=_heuristic) if len(dist) >= 20 else None  # (smaller: not worth a thread)
    if th is not None:
        th.start()
    try:
        S = tspgpu.Search(ctx, dist, shard=rank, nshards=world, depth=depth)
    finally:
        if th is not None:
            th.join()
    if "v" not in heur:
        _heuristic()  # (no thread, or it raised: here, so an error surfaces)
    try:
        if collective:
            # then the MIN of the ranks' costs: all starts' bound at 1/W of the host time
            ub_r, _ = heur["v"]
            word = tspgpu.cost_bits(ub_r, S.dtype) if ub_r is not None else (1 << 63) - 1
            ub = tspgpu.bits_cost(allmin2(word, 0)[0], S.dtype)
        else:
            ub, _ = heur["v"]
        S.set_bound(ub)
        t0 = time.perf_counter()
        exchanges = 0
        S.start()
        busy = 1
        while True:
            # up to exchange_every steps on this rank (while it has work), then
            # the exchange: incumbent MIN and "anyone still busy" (MIN of the
            # negated flag) in one all-reduce
            for _ in range(exchange_every):
                if not busy:
                    break
                busy = 1 if S.step() else 0
            inc, _, _ = S.counters()
            best, anybusy = allmin2(inc, -busy)
            exchanges += 1
            if best < inc:
                S.set_bound(tspgpu.bits_cost(best, S.dtype))
            if anybusy == 0:
                break
        inc, nodes, recs = S.counters()
        opt = allmin(inc)
        phases = 1

        def local_records():
            try:
                return S.records(opt), 0
            except tspgpu.TspGpuError as e:
                if e.code != -errno.EOVERFLOW:
                    raise
                return [], 1

        mine, lost = local_records()
        if allmin(-lost) < 0:
            # some rank lost records: search again with the optimum as the bound,
            # so only optimal tours are recorded, in a buffer of the needed size
            phases = 2
            S.reset_records(int(min(max(recs, 1 << 16), 1 << 22)))
            S.set_bound(tspgpu.bits_cost(opt, S.dtype))
            S.run_all()
            # the device node counter is cumulative over both phases (start does
            # not reset it), so it already holds phase 1 + phase 2
            _, nodes, recs = S.counters()
            mine, lost = local_records()
            if allmin(-lost) < 0:
                # too many optimal tours to enumerate (coincident cities): the DP
                # (K1-wide on this rank's GPU) gives tsp()'s tour directly for n <= 31
                if S.n > 31:
                    raise tspgpu.TspGpuError(-errno.EOVERFLOW, "solve_sharded")
                c, t, _ = ctx.solve_instance(np.asarray(dist, dtype=np.float64))
                cost = float(c) if S.dtype == tspgpu.F64 else int(c)
                stats = {"nodes": int(nodes), "rank_nodes": int(nodes), "optimal_tours": 0, "depth": S.depth,
                         "items": S.items, "phases": phases, "fallback": 1, "kernel_ms": S.timing()[0],
                         "wall_s": time.perf_counter() - t0, "exchanges": exchanges, "world": world,
                         "backend": backend}
                return cost, t, stats
        blob = np.frombuffer(b"".join(bytes(r) for r in mine), dtype=np.uint8) if mine else np.zeros(0, np.uint8)
        if collective:
            parts = [None] * world
            tdist.all_gather_object(parts, blob, group=group)
            node_t = _word_tensor(int(nodes), device)
            tdist.all_reduce(node_t, op=tdist.ReduceOp.SUM, group=group)
            total_nodes = int(node_t.item())
        else:
            parts, total_nodes = [blob], nodes
        rsz = ctypes_sizeof_record()
        allrec = []
        for p in parts:
            for i in range(0, len(p), rsz):
                allrec.append(tspgpu.TourRecord.from_buffer_copy(bytes(p[i:i + rsz])))
        cost = tspgpu.bits_cost(opt, S.dtype)
        tour = tspgpu.select_tour(dist, allrec, cost)
        wall = time.perf_counter() - t0
        kernel_ms, rounds = S.timing()
        stats = {"nodes": total_nodes, "rank_nodes": int(nodes), "optimal_tours": len(allrec), "depth": S.depth,
                 "items": S.items, "phases": phases, "fallback": 0, "kernel_ms": kernel_ms, "rounds": rounds,
                 "wall_s": wall,
                 "exchanges": exchanges, "exchange_every": exchange_every, "world": world, "backend": backend}
        return cost, tour, stats
    finally:
        S.close()


def ctypes_sizeof_record() -> int:
    import ctypes

    return ctypes.sizeof(tspgpu.TourRecord)
