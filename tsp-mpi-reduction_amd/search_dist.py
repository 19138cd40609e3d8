"""Multi-GPU driver of K2 (one process per GPU, torch.distributed).

One instance is split over the ranks of a process group: rank r searches the
seed prefixes p with p mod W == r (libtspgpu's static shard), as ONE chained
device run (every frontier level enqueued back to back, one synchronisation)
or, for searches too large to chain, step by step with an all-reduce(MIN) of
the 64-bit incumbent word (IEEE bits of the f64 cost or the integer cost;
both order like signed int64 for the non-negative costs the ABI accepts)
every few steps, so every GPU prunes with the best tour found anywhere.  At
the end: all-reduce(MIN) of the incumbent = the optimum, then all-reduce(MIN)
of each rank's device tie key at that cost (the reverse-lex least optimal
tour it found; w0, then w1 among its holders), certified once, on rank 0
(tspgpu_tie_tour_records from its own optimal records at world 1, else
tspgpu_tie_tour), and broadcast — one more collective, counted in the stats'
`collectives` — the same tour as tsp() / K1 on one GPU, SURVEY.md §8(e).
Records are gathered only when the certificate cannot be given.

With the "nccl" backend (RCCL on ROCm) the exchanges are device all-reduces
over xGMI; "gloo" runs the same logic over host tensors (CPU tests, or several
ranks sharing one GPU).  This replaces the reference's hand-rolled binary
MPI_Send/MPI_Recv tree (tsp.cpp:52-134) for the one step of the search that
needs a reduction: picking the global best tour (tsp.cpp:483-499's closing
min and its tie rule, across shards).
"""
from __future__ import annotations

import atexit
import errno
import os
import threading
import time

import numpy as np

import tspgpu


_COMM_LIB = None


def comm_lib():
    """libtspcomm (include/tspcomm.h): the RCCL communicator and the
    in-stream incumbent exchange hook; loaded only by multi-GPU drivers."""
    global _COMM_LIB
    if _COMM_LIB is None:
        import ctypes

        path = os.path.join(os.path.dirname(tspgpu.LIB_PATH), "libtspcomm.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build it (make -C tsp-mpi-reduction_amd)")
        L = ctypes.CDLL(path)
        vp, ip = ctypes.c_void_p, ctypes.c_int
        L.tspcomm_unique_id.argtypes = [ctypes.c_char_p, ip]
        L.tspcomm_create.argtypes = [ctypes.c_char_p, ip, ip, ip, ctypes.POINTER(vp)]
        L.tspcomm_destroy.argtypes = [vp]
        L.tspcomm_hook_stats.argtypes = [vp, ctypes.POINTER(ip), ctypes.POINTER(ip), ip]
        L.tspcomm_allreduce_min_u64.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ip, vp]
        _COMM_LIB = L
    return _COMM_LIB


class RcclComm:
    """An RCCL communicator over the ranks of a torch.distributed group
    (rank 0's ncclUniqueId broadcast over the group), for the in-stream
    incumbent exchange: `native_hook` is the (function, user) pair that
    tspgpu_search_chain calls between levels (tspcomm_level_hook: an
    ncclAllReduce MIN of the device incumbent word on the search's stream)."""

    def __init__(self, group, rank: int, world: int, device_index: int):
        import ctypes

        import torch
        import torch.distributed as tdist

        L = comm_lib()
        nb = L.tspcomm_unique_id_bytes()
        uid = ctypes.create_string_buffer(nb)
        if rank == 0:
            rc = L.tspcomm_unique_id(uid, nb)
            if rc:
                raise tspgpu.TspGpuError(rc, "tspcomm_unique_id")
        dev = torch.device("cuda", device_index) if tdist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor(list(uid.raw), dtype=torch.uint8, device=dev)
        src = tdist.get_global_rank(group, 0) if group is not None else 0
        tdist.broadcast(t, src=src, group=group)
        raw = bytes(t.cpu().tolist())
        h = ctypes.c_void_p()
        rc = L.tspcomm_create(raw, world, rank, device_index, ctypes.byref(h))
        if rc:
            raise tspgpu.TspGpuError(rc, "tspcomm_create")
        self.handle = h
        self.native_hook = (ctypes.cast(L.tspcomm_level_hook, ctypes.c_void_p).value, h)

    def hook_stats(self, reset: bool = True):
        """(hooks enqueued, hooks that failed to enqueue) since the last reset."""
        import ctypes

        c, e = ctypes.c_int(), ctypes.c_int()
        comm_lib().tspcomm_hook_stats(self.handle, ctypes.byref(c), ctypes.byref(e), int(reset))
        return c.value, e.value

    def close(self):
        if self.handle:
            comm_lib().tspcomm_destroy(self.handle)
            self.handle = None


_COMMS = {}


def _group_ranks(group):
    """The group's members as global ranks (its identity for the cache: id()
    of a freed subgroup can be reused by a new group with other members)."""
    import torch.distributed as tdist

    if group is None:
        return tuple(range(tdist.get_world_size()))
    return tuple(tdist.get_global_rank(group, r) for r in range(tdist.get_world_size(group)))


def rccl_comm(group, rank: int, world: int, device_index: int) -> RcclComm:
    """The process's communicator for this group and device (created once:
    ncclCommInitRank costs far more than a search).  Keyed on the group's
    global rank list and the process-group object, which the cache keeps
    alive (so its id is never reused: a re-initialised torch.distributed or a
    new subgroup gets its own communicator), and the device."""
    import torch.distributed as tdist

    pg = group if group is not None else tdist.group.WORLD
    key = (_group_ranks(group), id(pg), rank, world, device_index)
    ent = _COMMS.get(key)
    if ent is None or not ent[1].handle:
        ent = _COMMS[key] = (pg, RcclComm(group, rank, world, device_index))
    return ent[1]


def close_comms():
    """Destroy every cached RCCL communicator (ncclCommDestroy); called at
    exit, and safe to call before torch.distributed.destroy_process_group."""
    while _COMMS:
        _, (_, c) = _COMMS.popitem()
        try:
            c.close()
        except Exception:  # (at interpreter exit the library may be gone)
            pass


atexit.register(close_comms)


_I64_MAX = (1 << 63) - 1


def _key_i64(u: int) -> int:
    """u64 -> int64, order-preserving (torch all-reduce MIN is signed)."""
    v = (u ^ (1 << 63)) & ((1 << 64) - 1)
    return v - (1 << 64) if v >= (1 << 63) else v


def _key_u64(v: int) -> int:
    return ((v + (1 << 64)) % (1 << 64)) ^ (1 << 63)


def solve_sharded(ctx, dist, group=None, depth: int = 0, device=None, exchange_every: int | None = None,
                  exchange_levels: int = 2, bound: str | None = None):
    """Search one instance over the ranks of `group` (None: the default group,
    or a single process when torch.distributed is not initialised).

    1. The initial bound.  bound="device" (the default): the search's create
       launch computes it on the GPU (nearest neighbour + 2-opt from spread
       start cities, TSPGPU_SEARCH_DEVICE_BOUND) — the same on every rank, no
       host heuristic and no collective; round 6: the host multi-start took
       0.6-0.8 ms of a 1.7-1.9 ms 32-city solve.  bound="host": the host
       multi-start tour; from 20 cities each rank runs 1/W of the starts and
       the ranks all-reduce MIN, below every rank computes the same
       four-start bound itself.
    2. Each rank runs its shard as ONE device chain (tspgpu_search_chain: the
       seeds, every frontier level and the tail fold back to back, one
       synchronisation that also reads back the counters and the shard's tie
       slot at its incumbent), and every `exchange_levels` levels the
       incumbent is exchanged INSIDE the chain: with the "nccl" backend an
       RCCL all-reduce MIN of the device word enqueued on the search's stream
       between two levels (libtspcomm's hook, no host round trip); with gloo
       (CPU tests, ranks sharing a GPU) a host all-reduce MIN at the level
       boundary.  The hook count is the same on every rank.
    3. The winner (MIN of the cost, then MIN of the
       reverse-lex key among the holders of that cost): when every shard
       finished its chain, ONE all-gather of 7-word records (incumbent,
       chained, tie slot w0/w1/found/overflow, nodes) and the same
       lexicographic MIN on every rank; otherwise the stepwise search with one
       all-reduce MIN of (incumbent, -busy) every `exchange_every` steps
       (default 4; the same count on every rank, so the collectives pair up)
       followed by all-reduce MIN of w0 (ranks without one send the maximum)
       and of w1 among its holders.  Rank 0 certifies the winning key
       (tspgpu_tie_tour_gpu) and broadcasts the result — one more collective
       in stats["collectives"] — so every rank takes the same branch:
       tsp()'s tour with no record leaving any rank.
       Only when a tie table overflowed or the certificate fails do the ranks
       gather their optimal records for the host tie rule (a second search
       first if records were lost).

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
    ncoll = [0]

    def allmin(vals):
        if not collective:
            return [int(v) for v in vals]
        t = torch.tensor(vals, dtype=torch.int64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MIN, group=group)
        ncoll[0] += 1
        return [int(x) for x in t.tolist()]

    exchange_every = max(1, int(exchange_every or 4))

    def allgather(vals):
        """Every rank's record (a list of int64) -> [record of rank 0, ...]."""
        t = torch.tensor(vals, dtype=torch.int64, device=device)
        if not collective:
            return [[int(x) for x in t.tolist()]]
        parts = [torch.empty_like(t) for _ in range(world)]
        tdist.all_gather(parts, t, group=group)
        ncoll[0] += 1
        return [[int(x) for x in p.tolist()] for p in parts]

    # the multi-start tour.  From 20 cities it is split over the ranks (start
    # cities r, r+W, ...; all-reduce MIN of the costs) and computed on a thread
    # while the search is created (ctypes releases the GIL); below, every rank
    # computes the same four-start bound itself (microseconds; no collective)
    bound = bound or os.environ.get("TSPGPU_SHARDED_BOUND", "device")
    if bound not in ("device", "host"):
        raise ValueError(f"bound must be 'device' or 'host', not {bound!r}")
    dev_bound = bound == "device"
    split = not dev_bound and collective and world > 1 and len(dist) >= 20
    heur = {}

    def _heuristic():
        heur["v"] = tspgpu.heuristic_tour(dist, first=rank, step=world) if split else tspgpu.heuristic_tour(dist)

    # host phase clock (stats["host_phases_ms"]): where a rank's wall time goes
    ph, ph_t = {}, [time.perf_counter()]

    def mark(name):
        t = time.perf_counter()
        ph[name] = ph.get(name, 0.0) + (t - ph_t[0]) * 1e3
        ph_t[0] = t

    th = threading.Thread(target=_heuristic) if not dev_bound and len(dist) >= 20 else None  # (smaller: no thread)
    if th is not None:
        th.start()
    try:
        S = tspgpu.Search(ctx, dist, shard=rank, nshards=world, depth=depth, device_bound=dev_bound)
    finally:
        if th is not None:
            th.join()
    if not dev_bound and "v" not in heur:
        _heuristic()  # (no thread, or it raised: here, so an error surfaces)
    mark("create_and_heuristic")
    try:
        if split:
            ub_r, _ = heur["v"]
            word = tspgpu.cost_bits(ub_r, S.dtype) if ub_r is not None else _I64_MAX
            ub = tspgpu.bits_cost(allmin([word])[0], S.dtype)
            S.set_bound(ub)
        elif not dev_bound:
            ub, _ = heur["v"]
            S.set_bound(ub)
        mark("bound")
        t0 = time.perf_counter()
        two = S.n - 1 > 20
        exchanges = 0
        # the periodic incumbent exchange inside the chain (north_star: "the
        # incumbent bound is exchanged periodically")
        hooks = 0
        if backend == "nccl":
            comm = rccl_comm(group, rank, world, device.index if device.index is not None else 0)
            comm.hook_stats(reset=True)
            chained = S.chain(exchange_levels, native_hook=comm.native_hook)
            hooks, herr = comm.hook_stats(reset=True)
            if herr:
                raise tspgpu.TspGpuError(-errno.EIO, f"{herr} in-stream RCCL exchanges failed to enqueue")
        elif collective:
            nh, herr = [0], []

            def host_exchange(_stream, _word):
                # (gloo: the word through the host at the level boundary —
                # counters synchronises the stream up to here).  ctypes drops
                # an exception raised in a callback, so a failing rank would
                # skip its all-reduce while the others block in theirs: every
                # call joins the collective (with the neutral maximum when
                # its own word is unavailable) and the error is raised after
                # the chain returns.
                nh[0] += 1
                try:
                    cur = S.counters()[0] if not herr else _I64_MAX
                except Exception as e:  # noqa: BLE001 (re-raised below)
                    herr.append(e)
                    cur = _I64_MAX
                best = allmin([cur])[0]
                if not herr and best < cur:
                    try:
                        S.set_bound(tspgpu.bits_cost(best, S.dtype))
                    except Exception as e:  # noqa: BLE001
                        herr.append(e)

            chained = S.chain(exchange_levels, hook=host_exchange)
            hooks = nh[0]
            if herr:
                raise herr[0]
        else:
            chained = S.chain()
        mark("chain")
        inc, nodes, recs = S.counters()  # (a finished chain: from its own readback)
        # Fast path, every rank one finished chain: ONE collective.  Each rank
        # contributes (incumbent, chained, its tie slot at that incumbent,
        # nodes); the optimum is the MIN of the incumbents, the winner the
        # (w0, w1)-MIN over the ranks that hold a tour of that cost — the
        # all-reduce MIN of the cost and then of the key in
        # one all-gather of 7-word records, the same MIN computed on every rank.
        f, w0, w1, ovf = S.tie_slot(inc) if chained else (False, 0, 0, False)
        rec = allgather([inc, int(chained), int(f), _key_i64(w0) if f else _I64_MAX,
                         _key_i64(w1) if f and two else _I64_MAX, int(ovf), int(nodes)])
        exchanges = 1 + hooks
        fast = all(r[1] for r in rec)
        if fast:
            opt = min(r[0] for r in rec)
            total_nodes = sum(r[6] for r in rec)
            at_opt = [r for r in rec if r[0] == opt]  # (only a rank at the optimum can hold an optimal tour)
            holders = [r for r in at_opt if r[2]]
            nov = -1 if any(r[5] for r in at_opt) else 0
            K0, K1 = min((r[3], r[4]) for r in holders) if holders else (_I64_MAX, _I64_MAX)
        else:
            # some shard was too large to chain: step by step, one all-reduce
            # MIN of (incumbent, -busy) every exchange_every steps, the same
            # count on every rank (ranks whose chain finished only join)
            busy, exchanges = 0, hooks  # (the in-chain exchanges, then the loop's)
            if not chained:
                S.start()
                busy = 1
            while True:
                for _ in range(exchange_every):
                    if not busy:
                        break
                    busy = 1 if S.step() else 0
                inc, _, _ = S.counters()
                best, anybusy = allmin([inc, -busy])
                exchanges += 1
                if best < inc:
                    S.set_bound(tspgpu.bits_cost(best, S.dtype))
                if anybusy == 0:
                    break
            opt = best  # (the last exchange: every rank finished, so the MIN is the optimum)
            _, nodes, recs = S.counters()
            total_nodes = None
            # the device tie rule across ranks: MIN of w0, then of w1 among its holders
            found, w0, w1, ovf = S.tie_slot(opt) if inc <= opt else (False, 0, 0, False)
            k0 = _key_i64(w0) if found else _I64_MAX
            K0, nov = allmin([k0, -int(ovf)])
            K1 = 0
            if two:
                (K1,) = allmin([_key_i64(w1) if found and k0 == K0 else _I64_MAX])
        cost = tspgpu.bits_cost(opt, S.dtype)
        mark("winner")
        tie, tour = 0, None
        if nov == 0 and K0 != _I64_MAX:
            # certified ONCE, on rank 0, and broadcast: every rank then takes
            # the same branch below (a certificate that failed on one rank
            # only — ENOMEM on a shared GPU — would otherwise split the ranks
            # between the record gather's collectives and returning)
            rc, t = -errno.EAGAIN, np.zeros(S.n + 1, dtype=np.int32)
            if rank == 0:
                w = (_key_u64(K0), _key_u64(K1) if two else 0, cost)
                # one rank holds every record: the certificate's prefix minima
                # come from its optimal records (tspgpu_tie_tour_records), no
                # prefix DP; several ranks (records spread) or lost records:
                # the DP on this rank's GPU
                recs_opt = None
                if world == 1 and fast:
                    try:
                        recs_opt = S.records(opt)
                    except tspgpu.TspGpuError:
                        recs_opt = None
                if recs_opt:
                    rc, t = tspgpu.tie_tour_records(ctx, dist, *w, recs_opt)
                else:
                    rc, t = tspgpu.tie_tour_gpu(ctx, dist, *w) if ctx is not None else tspgpu.tie_tour(dist, *w)
            if collective:
                buf = torch.tensor([1 if rc == 0 else 0, *[int(x) for x in t]], dtype=torch.int64, device=device)
                src = tdist.get_global_rank(group, 0) if group is not None else 0
                tdist.broadcast(buf, src=src, group=group)
                ncoll[0] += 1
                vals = [int(x) for x in buf.tolist()]
                rc, t = (0 if vals[0] else -errno.EAGAIN), np.asarray(vals[1:], dtype=np.int32)
            if rc == 0:
                tie, tour = 1, t
        mark("certificate")
        phases, fallback, gathered, n_opt = 1, 0, 0, 0
        if not tie:
            tour, phases, fallback, nodes, n_opt = _records_winner(S, ctx, dist, opt, recs, nodes, allmin,
                                                                  collective, group)
            gathered = 1
        if total_nodes is None or phases == 2 or fallback:
            # (stepwise path: one SUM; phases 2: _records_winner summed phase 1 + 2 over the ranks; the
            # K1-wide fallback reports this rank's nodes)
            if phases == 1 and not fallback and collective:
                node_t = torch.tensor([int(nodes)], dtype=torch.int64, device=device)
                tdist.all_reduce(node_t, op=tdist.ReduceOp.SUM, group=group)
                ncoll[0] += 1
                total_nodes = int(node_t.item())
            else:
                total_nodes = int(nodes)
        wall = time.perf_counter() - t0
        kernel_ms, rounds = S.timing()
        mark("records_and_stats")
        stats = {"nodes": total_nodes, "rank_nodes": int(S.counters()[1]),
                 "optimal_tours": n_opt, "depth": S.depth,
                 "items": S.items, "phases": phases, "fallback": fallback, "kernel_ms": kernel_ms, "rounds": rounds,
                 "wall_s": wall, "tie": tie, "record_gather": gathered, "chained": int(chained),
                 "collectives": ncoll[0], "exchanges": exchanges, "hooks": hooks, "exchange_levels": exchange_levels,
                 "exchange_every": exchange_every, "world": world,
                 "backend": backend, "host_phases_ms": ph, "bound": bound}
        return cost, tour, stats
    finally:
        S.close()


def _records_winner(S, ctx, dist, opt, recs, nodes, allmin, collective, group):
    """Fallback winner: every rank's records at the optimum gathered for the
    host tie rule (a second search first when some rank lost records; K1-wide
    when too many tours tie).  -> (tour, phases, fallback, nodes, |O|)."""
    import torch
    import torch.distributed as tdist

    def local_records():
        try:
            return S.records(opt), 0
        except tspgpu.TspGpuError as e:
            if e.code != -errno.EOVERFLOW:
                raise
            return [], 1

    phases = 1
    mine, lost = local_records()
    if allmin([-lost])[0] < 0:
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
        if allmin([-lost])[0] < 0:
            # too many optimal tours to enumerate (coincident cities): the DP
            # (K1-wide on this rank's GPU) gives tsp()'s tour directly for n <= 31
            if S.n > 31:
                raise tspgpu.TspGpuError(-errno.EOVERFLOW, "solve_sharded")
            _, t, _ = ctx.solve_instance(np.asarray(dist, dtype=np.float64))
            return t, phases, 1, nodes, 0
    blob = np.frombuffer(b"".join(bytes(r) for r in mine), dtype=np.uint8) if mine else np.zeros(0, np.uint8)
    total_nodes = nodes
    if collective:
        parts = [None] * tdist.get_world_size(group)
        tdist.all_gather_object(parts, blob, group=group)
        if phases == 2:
            dev = torch.device("cpu") if tdist.get_backend(group) != "nccl" else \
                torch.device("cuda", torch.cuda.current_device())
            t = torch.tensor([int(nodes)], dtype=torch.int64, device=dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=group)
            total_nodes = int(t.item())
    else:
        parts = [blob]
    rsz = ctypes_sizeof_record()
    allrec = []
    for p in parts:
        for i in range(0, len(p), rsz):
            allrec.append(tspgpu.TourRecord.from_buffer_copy(bytes(p[i:i + rsz])))
    tour = tspgpu.select_tour(dist, allrec, tspgpu.bits_cost(opt, S.dtype))
    return tour, phases, 0, total_nodes, len(allrec)


def ctypes_sizeof_record() -> int:
    import ctypes

    return ctypes.sizeof(tspgpu.TourRecord)
