#!/usr/bin/env python3
"""Benchmark of the hot path: exact 16-city block search on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 16]
                    [--scaling strong|weak] [--global-blocks G] [--blocks-per-gpu B]

One STEP = one pass of K1 (the batched Held-Karp forward kernel + its
backtracking kernel, in launches of at most 16384 blocks) over this rank's
shard of blocks, inputs already resident in HBM.  The default is STRONG
scaling along the reference's own axis (tsp.cpp:159-195, 318-345): one fixed
instance `./tsp n G 1000 1000` (the reference's generator, srand(0);
G = 65536 by default) whose blocks the N ranks split with the reference's
per-rank counts, contiguously; `--scaling weak` gives every rank a fixed
`--blocks-per-gpu` shard instead, and the line carries the other form as
`other_scaling`.  There is no data-path collective: a gloo process group
provides the barriers and the max-over-ranks of the timed region
(measurement only).

`python bench.py --gpus N` without a launcher starts the N ranks itself (a
torch.distributed.run child; this parent never touches the GPU); under
torchrun (WORLD_SIZE set) each process is one rank, on GPU LOCAL_RANK.

`value` = Held-Karp DP relaxations (one (S,k,m) extension G[S\\k][m] + d[m][k]
with its min, tsp.cpp:457-470; N(N-1)2^(N-2) per block) of all ranks / max
wall time.  The K2 branch-and-bound probes report B&B search nodes in their
own keys (never mixed with relaxations).  Rank 0 prints ONE JSON line.

The GPU is driven only through libtspgpu's C ABI (device buffers, stream and
HIP-event timer included), so the HIP events sit on the stream the kernel runs
on.  torch is used only for torch.distributed.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import shutil
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "tsp-mpi-reduction_amd")
sys.path.insert(0, PKG)
import tspgpu  # noqa: E402  (lazy: loads libtspgpu on first use, no HIP call at import)

METRIC = "search nodes/sec (whole node) + time-to-optimal tour, 16-city, 1/2/4/8 GPU"
UNIT = "Held-Karp DP relaxations/s"
HBM_PEAK = 8.0e12  # B/s, MI355X_MICROARCH.md chip table (spec)
# VALU lane-instruction rates at the 2.4 GHz spec clock (MI355X_MICROARCH.md
# chip table: 256 CUs x 4 SIMDs, 157.3 TFLOPS f32 vector = 32 lanes/clk/SIMD
# x 2 for FMA): 32-bit integer ops at the f32 rate, f64 add/min at half of it
VALU_SPEC_I32 = 256 * 4 * 32 * 2.4e9  # 78.6 T lane-instructions/s
VALU_SPEC_F64 = 256 * 4 * 16 * 2.4e9  # 39.3 T lane-instructions/s
KERNEL_NAMES = {5: "hk_tiled_kernel", 6: "hk_sub_kernel"}  # K1 variant -> kernel symbol (others: heldkarp_kernel)
UBENCH = os.path.join(PKG, "bin", "ubench")
TSP_BIN = os.path.join(PKG, "bin", "tsp")


def kernel_name(variant):
    return KERNEL_NAMES.get(variant, "heldkarp_kernel")


def host_lib():
    import ctypes

    L = ctypes.CDLL(tspgpu.HOST_LIB_PATH)
    L.tsphost_generate.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(tspgpu.City)]
    return L


class Shard:
    """Cities of `./tsp n blocks_total grid grid` (tsp.cpp:373-403), blocks [lo, hi),
    kept as the C array the ABI takes."""

    def __init__(self, n, blocks_total, lo, hi, grid=1000):
        L = host_lib()
        full = (tspgpu.City * (n * blocks_total))()
        L.tsphost_generate(n, blocks_total, grid, grid, full)
        self.n, self.B, self.lo, self.hi = n, hi - lo, lo, hi
        self.arr = (tspgpu.City * (n * self.B)).from_buffer_copy(
            memoryview(full).cast("B")[lo * n * 24:hi * n * 24])

    def block(self, b):
        return [(self.arr[b * self.n + j].id, self.arr[b * self.n + j].x, self.arr[b * self.n + j].y)
                for j in range(self.n)]

    def distances(self):
        """Host libm distances, bit-exact with computeDistanceMatrix."""
        return tspgpu.distance_matrix_array(self.arr, self.n, self.B)


def shard_bounds(rank, world, per_rank):
    """Contiguous shard of the global instance owned by `rank` (weak scaling)."""
    return rank * per_rank, (rank + 1) * per_rank


def reference_counts(blocks, world):
    """Blocks per rank as the reference deals them (tsp.cpp:167-171: block
    b = B..1 goes to rank b mod P), in rank order."""
    cnt = [0] * world
    for b in range(blocks, 0, -1):
        cnt[b % world] += 1
    return cnt


def strong_bounds(rank, world, blocks):
    """Contiguous shard [lo, hi) of a FIXED global instance of `blocks` blocks
    owned by `rank` (strong scaling): the reference's per-rank counts, ranks
    in order (tsp.cpp:173-191 sends consecutive blocks to rank 0, 1, ...)."""
    cnt = reference_counts(blocks, world)
    lo = sum(cnt[:rank])
    return lo, lo + cnt[rank]


class Group:
    """Barrier + max/sum/gather over ranks (gloo; measurement only, the block
    path has no data collective)."""

    def __init__(self, world):
        self.dist = None
        if world > 1:
            import torch.distributed as dist

            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x, op):
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def allmax(self, x):
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist else x

    def allsum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist else x

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(out, obj)
        return out


def timed_steps(step, sync, group, warmup, steps, begin=None, end=None):
    """W untimed steps, then exactly K steps bracketed by barrier + device sync
    on both sides; `begin`/`end` run right inside the timed region (the HIP
    event pair).  Returns (max-over-ranks wall seconds, local wall seconds)."""
    for _ in range(warmup):
        step()
    sync()
    group.barrier()
    sync()
    t0 = time.perf_counter()
    if begin:
        begin()
    for _ in range(steps):
        step()
    if end:
        end()
    sync()
    group.barrier()
    wall = time.perf_counter() - t0
    return group.allmax(wall), wall


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv, gpus):
    """`bench.py --gpus N` with no launcher: start the N ranks as a child
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) and
    return its exit status.  This process never initialises the GPU, and it
    starts the launcher as a child instead of exec'ing it."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    return subprocess.call(cmd, env=env)


# --------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1): the reference itself, then the oracle port
# --------------------------------------------------------------------------
def host_cpus():
    """CPUs this process may use: the affinity set, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def find_mpirun():
    for c in (shutil.which("mpirun"), "/opt/conda/bin/mpirun"):
        if c and os.path.exists(c):
            return c
    return None


def cpu_baseline(n, max_ranks=None):
    """The reference's own program timed on this host's cores: `mpirun -np P
    ./tsp n P 1000 1000` with P = the usable cores (one 16-city block per
    rank, the reference's own distribution, tsp() and reduction tree; the
    binary is built from /root/reference at -O0 by oracle/Makefile, nothing
    else from the reference is used).  value = P blocks' DP relaxations / the
    program's own printed milliseconds (tsp.cpp:275-276, 360-363).  Without
    mpirun: one reference tsp() per process (oracle/_ref/ref_harness timeone)
    on every core; without the reference binaries: the C oracle port."""
    cores = host_cpus()
    P = cores if max_ranks is None else min(cores, max_ranks)
    relax = tspgpu.relaxations_per_block(n)
    ref_tsp = os.path.join(ROOT, "oracle", "_ref", "tsp")
    ref_h = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    mpirun = find_mpirun()
    base = {"unit": UNIT, "cores": P, "cpu_model": cpu_model(), "host_cpus_usable": cores}
    if mpirun and os.path.exists(ref_tsp):
        try:
            env = dict(os.environ, OMP_NUM_THREADS="1")
            cmd = [mpirun, "-np", str(P), ref_tsp, str(n), str(P), "1000", "1000"]
            t0 = time.perf_counter()
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
            wall = time.perf_counter() - t0
            m = re.search(r"TSP ran in (\d+) ms for (\d+) cities and the trip cost ([0-9.]+)", p.stdout)
            if p.returncode == 0 and m:
                ms = int(m.group(1))
                return dict(base, value=P * relax / (ms * 1e-3), kind="reference", launcher="mpirun",
                            sample=f"`{os.path.basename(mpirun)} -np {P} ./tsp {n} {P} 1000 1000` (the reference "
                                   f"program, MPICH, one {n}-city block per rank): the program's own clock "
                                   f"{ms} ms, process wall {wall:.2f} s, cost {m.group(3)}",
                            blocks_per_s=P / (ms * 1e-3), reference_ms=ms, wall_s=wall)
            sys.stderr.write(f"cpu_baseline: mpirun run failed rc={p.returncode}: {p.stderr[-300:]}\n")
        except Exception as e:  # noqa: BLE001 - fall through to the per-process harness
            sys.stderr.write(f"cpu_baseline: mpirun failed ({e})\n")
    if os.path.exists(ref_h):
        try:
            t0 = time.perf_counter()
            procs = [subprocess.Popen([ref_h, "timeone", str(n), str(P), "1000", "1000", str(i)],
                                      stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
                     for i in range(P)]
            outs = [p.communicate(timeout=600)[0] for p in procs]
            wall = time.perf_counter() - t0
            per = [float(ln.split()[2]) for o in outs for ln in o.splitlines() if ln.startswith("T ")]
            if len(per) == P and all(p.returncode == 0 for p in procs):
                return dict(base, value=P * relax / wall, kind="reference", launcher="per-process harness (no mpirun)",
                            sample=f"{P} blocks x {n} cities of `./tsp {n} {P} 1000 1000`, the reference's tsp() "
                                   f"(-O0) one block per process on {P} cores; {wall:.1f} s wall, median block "
                                   f"{statistics.median(per):.2f} s", blocks_per_s=P / wall)
        except Exception as e:  # noqa: BLE001
            sys.stderr.write(f"cpu_baseline: reference harness failed ({e}); using the oracle port\n")
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O

    shard = Shard(n, 64, 0, 64)
    d = shard.distances()
    t0 = time.perf_counter()
    k = 0
    while k < shard.B and time.perf_counter() - t0 < 20.0:
        O.solve_block(d[k])
        k += 1
    wall = time.perf_counter() - t0
    return dict(base, value=k * relax / wall, cores=1, kind="port", launcher="none",
                sample=f"{k} blocks x {n} cities, oracle array Held-Karp (-O2), 1 core, {wall:.1f} s",
                blocks_per_s=k / wall)


def cpu_optimized(n, seconds_budget=5.0):
    """A second, optimized CPU baseline beside the reference's own path
    (SURVEY.md §8(d)): the oracle's array Held-Karp (C, -O2, the same bits)
    on every usable host core (ctypes releases the GIL), on the same generated
    blocks.  Reported next to cpu_baseline, never as the headline."""
    import threading

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py as O

    cores = host_cpus()
    shard = Shard(n, max(256, 4 * cores), 0, max(256, 4 * cores))
    d = shard.distances()
    done = [0] * cores
    t0 = time.perf_counter()

    def work(w):
        b = w
        while b < shard.B and time.perf_counter() - t0 < seconds_budget:
            O.solve_block(d[b])
            done[w] += 1
            b += cores

    th = [threading.Thread(target=work, args=(w,)) for w in range(cores)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    k = sum(done)
    return {"value": k * tspgpu.relaxations_per_block(n) / wall, "unit": UNIT, "cores": cores,
            "kind": "port", "sample": f"{k} blocks x {n} cities, oracle array Held-Karp (C -O2) on {cores} threads, "
                                      f"{wall:.1f} s", "blocks_per_s": k / wall}


# --------------------------------------------------------------------------
# Time to optimal, the reference's own definition: process start -> final line
# --------------------------------------------------------------------------
def cli_wall(n, reps=3):
    """`bin/tsp n 1 1000 1000` (the drop-in program) as a child process: wall
    time from spawn to exit (process start, HIP init, generation, K1, merge,
    final line), best of `reps`, next to the ms the program prints itself
    (tsp.cpp:275-276, 360-363 measure from main's first line)."""
    if not os.path.exists(TSP_BIN):
        return {"error": "bin/tsp not built"}
    best = None
    env = dict(os.environ, TSP_STATS="1")
    st = re.compile(r"HIP runtime start-up ([0-9.]+) ms")
    for _ in range(reps):
        t0 = time.perf_counter()
        p = subprocess.run([TSP_BIN, str(n), "1", "1000", "1000"], capture_output=True, text=True, timeout=120,
                           env=env)
        wall = (time.perf_counter() - t0) * 1e3
        m = re.search(r"TSP ran in (\d+) ms for (\d+) cities and the trip cost ([0-9.]+)", p.stdout)
        if p.returncode != 0 or not m:
            return {"error": f"rc={p.returncode} {p.stderr[-200:]}"}
        q = st.search(p.stderr)
        rt = float(q.group(1)) if q else None
        if best is None or wall < best["process_wall_ms"]:
            # hip_runtime_startup_ms: the runtime's own initialisation inside the
            # program clock (hipGetDeviceCount's first call; the analogue of the
            # reference's MPI_Init, tsp.cpp:275-278), the rest is the drop-in's
            best = {"command": f"./tsp {n} 1 1000 1000", "process_wall_ms": wall, "program_ms": int(m.group(1)),
                    "hip_runtime_startup_ms": rt,
                    "program_ms_after_runtime_startup": int(m.group(1)) - rt if rt is not None else None,
                    "cost": m.group(3)}
    return best


# the merge-dominated runs, where mergeBlocks
# (tsp.cpp:202-269, O(L1*L2^2) through rotate) is the program; the reference's
# own times on the survey's 8-core Xeon
K3_CASES = ((4, 1024, 1, 7100), (4, 1024, 8, 30900), (8, 1024, 8, 237056))


def k3_merge(reps=2):
    """K3 (the GPU mergeBlocks) where it dominates: `bin/tsp n 1024 1000
    1000` with TSP_NPROCS=P, the program's own clock (tsp.cpp:275-276,
    360-363) and its TSP_STATS phase split (block search, merge), the final
    cost checked against the reference's (tests/golden/cli_large.json), next
    to the reference's measured time (237 s for ./tsp 8 1024
    on 8 ranks)."""
    if not os.path.exists(TSP_BIN):
        return {"error": "bin/tsp not built"}
    gold = {}
    try:
        with open(os.path.join(ROOT, "tests", "golden", "cli_large.json")) as f:
            for c in json.load(f)["data"]:
                gold[(tuple(c["args"]), c["P"])] = c["lines"][-1].rsplit(" ", 1)[1]
    except (OSError, KeyError, ValueError):
        pass
    pat = re.compile(r"TSP ran in (\d+) ms for (\d+) cities and the trip cost ([0-9.]+)")
    st = re.compile(r"block search ([0-9.]+) ms.*merge ([0-9.]+) ms, total ([0-9.]+) ms")
    out = {}
    for n, B, P, ref_ms in K3_CASES:
        env = dict(os.environ, TSP_NPROCS=str(P), TSP_STATS="1")
        for k in ("PMI_SIZE", "PMI_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_RANK"):
            env.pop(k, None)
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            p = subprocess.run([TSP_BIN, str(n), str(B), "1000", "1000"], capture_output=True, text=True,
                               timeout=300, env=env)
            wall = (time.perf_counter() - t0) * 1e3
            m, q = pat.search(p.stdout), st.search(p.stderr)
            if p.returncode != 0 or not m:
                best = {"error": f"rc={p.returncode} {p.stderr[-200:]}"}
                break
            r = {"program_ms": int(m.group(1)), "process_wall_ms": wall, "cost": m.group(3),
                 "block_search_ms": float(q.group(1)) if q else None, "merge_ms": float(q.group(2)) if q else None}
            if best is None or r["program_ms"] < best["program_ms"]:
                best = r
        if "cost" in best:
            g = gold.get(((n, B, 1000, 1000), P))
            best["reference_cost"] = g
            best["same_cost"] = g == best["cost"] if g else None
            best["reference_ms_survey_xeon"] = ref_ms
            best["speedup_vs_reference"] = ref_ms / max(best["program_ms"], 1)
        out[f"./tsp {n} {B} 1000 1000 P={P}"] = best
    return out


def reference_multiblock(n=16, blocks=8, procs=(1, 2, 4, 8)):
    """The reference's own multi-block runs beside the drop-in, on this box:
    `mpirun -np P ./tsp n B 1000 1000` (the reference, oracle/_ref/tsp, one
    core per rank) against `bin/tsp n B 1000 1000` for the same logical P —
    once as one process (TSP_NPROCS=P, every block in one batched launch) and
    once under the same `mpirun -np P` (a process per rank, each solving its
    share on the GPU).  Each time is the program's own clock, process start to
    the final line (tsp.cpp:275-276, 360-363), next to the launcher's wall; the
    final cost lines must agree.  BASELINE.md quotes the reference's 8-core
    Xeon times for `./tsp 16 8` at P = 1/2/4/8: 33.5 / 17.1 / 8.4 / 5.0 s."""
    ref = os.path.join(ROOT, "oracle", "_ref", "tsp")
    mpirun = find_mpirun()
    if not (mpirun and os.path.exists(ref) and os.path.exists(TSP_BIN)):
        return {"error": "needs mpirun, oracle/_ref/tsp and bin/tsp"}
    pat = re.compile(r"TSP ran in (\d+) ms for (\d+) cities and the trip cost ([0-9.]+)")

    def run(cmd, env):
        t0 = time.perf_counter()
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
        wall = time.perf_counter() - t0
        m = pat.search(p.stdout)
        if p.returncode != 0 or not m:
            return {"error": f"rc={p.returncode} {p.stderr[-200:]}"}
        return {"program_ms": int(m.group(1)), "process_wall_ms": wall * 1e3, "cost": m.group(3)}

    base_env = dict(os.environ, OMP_NUM_THREADS="1")
    base_env.pop("TSP_NPROCS", None)
    out = {"command": f"./tsp {n} {blocks} 1000 1000", "cpu_model": cpu_model(), "runs": {}}
    for P in procs:
        if P > host_cpus():
            continue
        args = [str(n), str(blocks), "1000", "1000"]
        r = {"reference_mpirun": run([mpirun, "-np", str(P), ref, *args], base_env),
             "dropin_one_process": run([TSP_BIN, *args], dict(base_env, TSP_NPROCS=str(P))),
             "dropin_mpirun": run([mpirun, "-np", str(P), TSP_BIN, *args], base_env)}
        costs = {v.get("cost") for v in r.values()}
        r["same_cost"] = len(costs) == 1 and None not in costs
        if "program_ms" in r["reference_mpirun"] and "program_ms" in r["dropin_one_process"]:
            r["speedup_program_clock"] = (r["reference_mpirun"]["program_ms"] /
                                          max(r["dropin_one_process"]["program_ms"], 1))
        out["runs"][f"P{P}"] = r
    return out


def scaling_probe(ctx, args, world, rank, group, n, relax):
    """The scaling form the headline does not use, on the same ranks: with
    --scaling strong every rank also solves its own fixed --blocks-per-gpu
    shard of `./tsp n blocks_per_gpu*N` (weak), with --scaling weak the ranks
    split one fixed --global-blocks instance (strong).  Same step, barriers
    and max-over-ranks as the headline; fewer steps."""
    if args.scaling == "strong":
        form, total = "weak", args.blocks_per_gpu * world
        lo, hi = shard_bounds(rank, world, args.blocks_per_gpu)
    else:
        form, total = "strong", args.global_blocks
        lo, hi = strong_bounds(rank, world, total)
    B = hi - lo
    d = Shard(n, total, lo, hi).distances()
    dd, dc, dt = ctx.upload(d), ctx.alloc(max(B, 1) * 8), ctx.alloc(max(B, 1) * (n + 1) * 4)
    steps = max(3, args.steps // 2)
    try:
        wall_max, _ = timed_steps(lambda: ctx.solve_device(dd, n, B, dc, dt, ctx.stream), ctx.synchronize,
                                  group, 1, steps)
    finally:
        for p_ in (dd, dc, dt):
            ctx.free(p_)
    return {"scaling": form, "value": total * steps * relax / wall_max, "unit": UNIT, "global_blocks": total,
            "blocks_this_rank": B, "steps": steps, "ms_per_step": wall_max / steps * 1e3}


# --------------------------------------------------------------------------
# K2 probes (branch-and-bound search nodes, their own unit)
# --------------------------------------------------------------------------
VALU_PEAK_SPEC = 256 * 4 * 16 * 2.4e9  # f64 lane-ops/s at 2.4 GHz (half-rate f64 on SIMD32)


def k2_exhaustive(ctx, n=14, reps=3):
    """BASELINE config 2: `./tsp 14 1 1000 1000` by exhaustive enumeration on
    one GPU (enum.hip: a lane per depth-7 prefix, its 720 completions folded in
    registers).  Roofline: VALU issue — one f64 add per partial path (node)
    plus one closing add and one min per tour."""
    d = Shard(n, 1, 0, 1).distances()[0]
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        cost, tour, st = tspgpu.search_solve(ctx, d, exhaustive=True)
        wall = (time.perf_counter() - t) * 1e3
        if best is None or wall < best[0]:
            best = (wall, cost, tour, st)
    wall, cost, tour, st = best
    sec = max(st["kernel_ms"] * 1e-3, 1e-12)
    tours = math.factorial(n - 1)
    ops = st["nodes"] + 2 * tours
    return {"instance": f"./tsp {n} 1 1000 1000 (block 0)", "cost": cost, "tour": [int(x) for x in tour],
            "time_to_optimal_ms": wall, "kernel_ms": st["kernel_ms"], "tours": tours,
            "tours_per_s": tours / sec, "bb_nodes": st["nodes"], "bb_nodes_per_s": st["nodes"] / sec,
            "roofline": {"bound": "valu", "achieved": ops / sec / 1e12, "peak": VALU_PEAK_SPEC / 1e12,
                         "unit": "T f64 lane-ops/s", "frac": ops / sec / VALU_PEAK_SPEC,
                         "note": "enum_kernel: (nodes + 2 x tours) algorithmic f64 ops / HIP-event kernel time"},
            "rounds": st["rounds"]}


TSPLIB_OPTIMA = {"burma14.tsp": 3323, "ulysses16.tsp": 6859, "gr17.tsp": 2085,
                 "ulysses22.tsp": 7013}  # published TSPLIB optima


def config4_tsplib(ctx, reps=3):
    """BASELINE config 4 on the real TSPLIB instances (tests/golden/tsplib):
    the DP over the whole GPU (K1-wide) and K2 in integer mode, time to the
    optimal tour (and B&B nodes), the cost checked against the published
    optimum.  K2 runs on all four: before its Held-Karp tree bound ulysses22
    took it 4.2e12 nodes and 7.9 s (profiles/r02/config4_tsplib.json) where
    the DP takes well under a millisecond."""
    out = {}
    for name, opt in TSPLIB_OPTIMA.items():
        _, d = tspgpu.read_tsplib(os.path.join(ROOT, "tests", "golden", "tsplib", name))
        n = int(d.shape[0])
        rec = {"n": n, "published_optimum": opt}
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            cost, tour, kms = ctx.solve_instance(d.astype(np.float64))
            wall = (time.perf_counter() - t) * 1e3
            if best is None or wall < best[0]:
                best = (wall, cost, tour, kms)
        assert best[1] == opt, f"{name}: DP {best[1]} != published optimum {opt}"
        rec["dp_k1_wide"] = {"cost": int(best[1]), "time_to_optimal_ms": best[0], "kernel_ms": best[3],
                             "tour": [int(x) for x in best[2]]}
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            cost, tour, st = tspgpu.search_solve(ctx, d)
            wall = (time.perf_counter() - t) * 1e3
            if best is None or wall < best[0]:
                best = (wall, cost, tour, st)
        wall, cost, tour, st = best
        assert cost == opt, f"{name}: K2 {cost} != published optimum {opt}"
        rec["k2_search"] = {"cost": int(cost), "time_to_optimal_ms": wall, "kernel_ms": st["kernel_ms"],
                            "bb_nodes_expanded": st["nodes"], "tour": [int(x) for x in tour]}
        out[name] = rec
    return out


def k2_instance(n, seed):
    """Config 5's extension instance: n uniform random cities in [0,1000)^2
    (seeded), libm distances like computeDistanceMatrix."""
    rng = np.random.default_rng(seed)
    xy = rng.uniform(0, 1000, size=(n, 2))
    return tspgpu.distance_matrix([[(i, xy[i, 0], xy[i, 1]) for i in range(n)]])[0]


def k2_group(world, local_rank):
    if world == 1:
        return None, "none"
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if ndev >= world:
        # one GPU per rank: the incumbent exchange is an RCCL all-reduce over xGMI
        torch.cuda.set_device(local_rank % ndev)
        return dist.new_group(backend="nccl"), "nccl"
    # ranks share a GPU (a rehearsal on a smaller box; RCCL wants one rank per
    # device) or no GPU: the same exchange over gloo
    return dist.new_group(backend="gloo"), "gloo"


def k2_single_instance(ctx, n, group, backend, world, reps=5):
    """K2 on the reference's own instance `./tsp n 1 1000 1000` (config 3's
    16 cities): time to the optimal tour and B&B nodes (sharded over the ranks
    with RCCL between rounds when N > 1)."""
    import search_dist

    d = Shard(n, 1, 0, 1).distances()[0]

    def best_of(fn):
        best = None
        for _ in range(reps):
            if group is not None:  # (the ranks start each search together)
                import torch.distributed as dist

                dist.barrier(group=group)
            t = time.perf_counter()
            cost, tour, st = fn()
            wall = (time.perf_counter() - t) * 1e3
            if best is None or wall < best[0]:
                best = (wall, cost, tour, st)
        return best

    sharded = best_of(lambda: search_dist.solve_sharded(ctx, d, group=group))
    if world == 1:
        wall, cost, tour, st = best_of(lambda: tspgpu.search_solve(ctx, d))
        st = dict(st, exchanges=0)
        assert cost == sharded[1] and list(tour) == list(sharded[2]), "native and sharded K2 disagree"
    else:
        wall, cost, tour, st = sharded
    return {"instance": f"./tsp {n} 1 1000 1000 (block 0)", "cost": cost, "time_to_optimal_ms": wall,
            "kernel_ms": st["kernel_ms"], "bb_nodes_expanded": st["nodes"],
            "bb_nodes_per_s": st["nodes"] / max(st["kernel_ms"] * 1e-3, 1e-12), "rounds": st["rounds"],
            "exchanges": st["exchanges"], "ranks": world, "exchange_backend": backend,
            "path": "tspgpu_search_solve (chained levels, one synchronisation)" if world == 1
            else "search_dist.solve_sharded",
            "python_exchange_loop_ms": sharded[0],
            "optimal_tours": st["optimal_tours"], "tour": [int(x) for x in tour],
            "device_tie_rule": {"used": int(st.get("tie", 0)), "records_agree": int(st.get("tie_checked", 0)),
                                "phases": int(st.get("phases", 1)), "fallback": int(st.get("fallback", 0)),
                                "record_gather": int(st.get("record_gather", 0)),
                                "chained": int(st.get("chained", 1)),
                                "collectives": int(st.get("collectives", 0))}}


def k2_strong_scaling(ctx, n, seed, group, backend, world, rank, reps=2):
    """Strong scaling of ONE instance over the N ranks (config 3/5 shape): the
    prefix space is sharded statically (prefix p -> rank p mod N), every rank
    runs its device queue in rounds and the 64-bit incumbent is all-reduced
    (MIN) between rounds over RCCL; the optimal records are gathered at the
    end for the DP tie rule.  time_to_optimal_ms = max over ranks of the
    solve's wall time (distances already on the host)."""
    import search_dist

    d = k2_instance(n, seed)
    best = None
    for _ in range(reps):
        if group is not None:
            import torch.distributed as dist

            dist.barrier(group=group)
        t = time.perf_counter()
        cost, tour, st = search_dist.solve_sharded(ctx, d, group=group)
        wall = (time.perf_counter() - t) * 1e3
        if best is None or wall < best[0]:
            best = (wall, cost, tour, st)
    wall, cost, tour, st = best
    return {"instance": f"{n} uniform random cities in [0,1000)^2, seed {seed} (config 5 shape)", "n": n,
            "ranks": world, "backend": backend, "cost": cost, "tour": [int(x) for x in tour],
            "rank_wall_ms": wall, "rank_kernel_ms": st["kernel_ms"], "rank_nodes": st["rank_nodes"],
            "bb_nodes_expanded": st["nodes"], "rounds": st.get("rounds"), "exchanges": st["exchanges"],
            "in_chain_exchanges": st.get("hooks", 0), "exchange_levels": st.get("exchange_levels"),
            "chained": st.get("chained"), "optimal_tours": st["optimal_tours"],
            "host_phases_ms": st.get("host_phases_ms"),
            "exchange": "RCCL all-reduce MIN of the device incumbent inside the chain every "
                        f"{st.get('exchange_levels')} levels (libtspcomm), then one all-gather" if backend == "nccl"
                        else ("host all-reduce MIN at level boundaries (gloo)" if world > 1 else "none (one rank)")}


# --------------------------------------------------------------------------
# Roofline inputs: live VALU peak and PMC passes (rank 0, N = 1)
# --------------------------------------------------------------------------
def valu_peaks():
    """Issue rates measured on this GPU by bin/ubench (the relaxation's own
    instruction mix: v_add_f64, v_cmp_lt_f64, v_cndmask_b32, v_min_f64)."""
    if not os.path.exists(UBENCH):
        return None
    p = subprocess.run(["timeout", "-k", "5", "60", UBENCH, "valu"], capture_output=True, text=True)
    if p.returncode != 0:
        return None
    out = {}
    for ln in p.stdout.splitlines():
        r = json.loads(ln)
        if "mix" in r:
            out[r["mix"]] = r["lane_ops_per_s"]
    return out


def _rocprof_pass(counters, n, blocks, kernel, tag, timeout=90, child=None, reduce="median"):
    """One rocprofv3 --pmc pass over a child run of this file: the K1 launch
    (--pmc-child) or, with child = [...], other child arguments.  `kernel`: a
    substring or a tuple of them; reduce "median" over the matching
    dispatches, or "sum"."""
    rocprof = shutil.which("rocprofv3")
    if not rocprof:
        return None, "rocprofv3 not found"
    d = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    shutil.rmtree(d, ignore_errors=True)
    child = child or ["--pmc-child", "--n", str(n), "--blocks-per-gpu", str(blocks)]
    cmd = ["timeout", "-s", "KILL", str(timeout), rocprof, "--pmc", *counters, "--output-format", "csv",
           "-d", d, "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), *child]
    p = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
    import collections
    import csv

    names = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    vals = collections.defaultdict(list)
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                with open(os.path.join(root, f)) as fh:
                    for row in csv.DictReader(fh):
                        if any(k in row.get("Kernel_Name", "") for k in names):
                            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if p.returncode != 0 or not vals:
        return None, f"rc={p.returncode} {p.stderr[-300:]}"
    agg = sum if reduce == "sum" else statistics.median
    return {k: agg(v) for k, v in vals.items()}, None


K2_KERNELS = ("prologue_kernel", "prologue1_kernel", "expand_kernel", "tail_kernel")
K2_PMC_SEARCHES = 4  # searches the K2 PMC child runs (counters are summed over them)


def k2_pmc(cus, peaks, nodes_per_search, kernel_ms):
    """SQ counters of the K2 search kernels (the reference's 16-city
    instance, K2_PMC_SEARCHES searches, counters summed and divided back per
    search): VALU instructions per B&B node, VALU active, and the VALU issue
    rate those kernels reach against the f64 add rate measured on this GPU."""
    sq, err = _rocprof_pass(SQ_PASS, 16, 1, K2_KERNELS, "k2_sq", child=["--pmc-child-k2"], reduce="sum")
    if not sq:
        return {"error": err}
    per = {k: v / K2_PMC_SEARCHES for k, v in sq.items()}
    lane_instr = per["SQ_INSTS_VALU"] * 64.0
    out = {"kernels": list(K2_KERNELS), "valu_wave_instructions_per_search": per["SQ_INSTS_VALU"],
           "valu_lane_instructions_per_node": lane_instr / max(nodes_per_search, 1),
           "waves_per_search": per["SQ_WAVES"], "sq_raw_per_search": per}
    peak = (peaks or {}).get("v_add_f64")
    if peak and kernel_ms:
        ach = lane_instr / (kernel_ms * 1e-3)
        out["roofline"] = {"bound": "valu (issue)", "achieved": ach / 1e12, "peak": peak / 1e12,
                           "unit": "T VALU lane-instructions/s", "frac": ach / peak,
                           "note": "VALU lane-instructions of the search kernels (PMC SQ_INSTS_VALU x 64) per search / "
                                   "the search's device time (device wall clock from the prologue's start to the "
                                   "readback kernel's, gaps included), "
                                   "against the f64 add issue rate (bin/ubench); "
                                   "a node costs valu_lane_instructions_per_node of them"}
    return out


def pmc_child_k2():
    ctx = tspgpu.Context(device=0)
    d = Shard(16, 1, 0, 1).distances()[0]
    for _ in range(K2_PMC_SEARCHES):
        tspgpu.search_solve(ctx, d)


SQ_PASS = ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU",
           "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE")
EA_PASS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_DRAM_sum")


def pmc_profile(n, blocks, cus, kernel):
    """rocprofv3 passes over the dominant kernel (one counter group per pass,
    MI355X_MICROARCH.md §rocprofv3 PMC slots):
      FETCH_SIZE, WRITE_SIZE — bytes at the L2's memory side (Infinity-Cache
        hits included; FETCH_SIZE x2: calibrated on 8-B loads, profiles/r02);
      TCC_EA0_{RD,WR}REQ[_DRAM] — the same requests split by whether DRAM
        served them, i.e. what HBM actually moved;
      SQ — VALU activity, instructions, LDS bank conflicts, occupancy."""
    out = {"blocks_per_launch": blocks}
    f, err = _rocprof_pass(("FETCH_SIZE",), n, blocks, kernel, "fetch")
    w, err2 = _rocprof_pass(("WRITE_SIZE",), n, blocks, kernel, "write")
    ea, err3 = _rocprof_pass(EA_PASS, n, blocks, kernel, "ea")
    sq, err4 = _rocprof_pass(SQ_PASS, n, blocks, kernel, "sq")
    if f and w:
        out["fabric_read_bytes"] = f["FETCH_SIZE"] * 1024 * 2
        out["fabric_write_bytes"] = w["WRITE_SIZE"] * 1024
    if ea:
        rd, rdd = ea.get("TCC_EA0_RDREQ_sum", 0), ea.get("TCC_EA0_RDREQ_DRAM_sum", 0)
        wr, wrd = ea.get("TCC_EA0_WRREQ_sum", 0), ea.get("TCC_EA0_WRREQ_DRAM_sum", 0)
        out["dram_read_frac"] = rdd / rd if rd else None
        out["dram_write_frac"] = wrd / wr if wr else None
        if "fabric_read_bytes" in out:
            out["hbm_bytes"] = (out["fabric_read_bytes"] * (out["dram_read_frac"] or 0) +
                                out["fabric_write_bytes"] * (out["dram_write_frac"] or 0))
        out["ea_raw"] = ea
    if sq and all(k in sq for k in SQ_PASS):
        cycles = sq["GRBM_GUI_ACTIVE"] / 8.0  # per XCD = kernel cycles
        simds = 4 * cus
        out.update({
            "valu_active_per_simd_cycle": 4.0 * sq["SQ_ACTIVE_INST_VALU"] / (simds * cycles),
            "valu_instructions_per_block": sq["SQ_INSTS_VALU"] / blocks,
            "lds_bank_conflict_cycles_over_lds_active": sq["SQ_LDS_BANK_CONFLICT"] / max(sq["SQ_ACTIVE_INST_LDS"], 1.0),
            "mean_resident_waves_per_cu": 4.0 * sq["SQ_WAVE_CYCLES"] / (cus * cycles),
            "sq_raw": sq,
        })
    errs = [e for e in (err, err2, err3, err4) if e]
    if errs:
        out["errors"] = errs
    return out


def pmc_child(args):
    ctx = tspgpu.Context(device=0)
    shard = Shard(args.n, args.blocks_per_gpu, 0, args.blocks_per_gpu)
    d = shard.distances()
    B, n = shard.B, args.n
    dd, dc, dt = ctx.upload(d), ctx.alloc(B * 8), ctx.alloc(B * (n + 1) * 4)
    for _ in range(3):
        ctx.solve_device(dd, n, B, dc, dt, ctx.stream)
    ctx.synchronize()


def plumbing(args, world, rank):
    """--plumbing (CPU, no GPU): the multi-rank orchestration alone — shard
    bounds of every rank, the barrier-bracketed region and the max over
    ranks — printed by rank 0 (tests/test_bench_cli.py)."""
    group = Group(world)
    if args.scaling == "strong":
        lo, hi = strong_bounds(rank, world, args.global_blocks)
        global_blocks = args.global_blocks
    else:
        lo, hi = shard_bounds(rank, world, args.blocks_per_gpu)
        global_blocks = args.blocks_per_gpu * world
    wall_max, wall = timed_steps(lambda: None, lambda: None, group, args.warmup, args.steps)
    shards = group.gather([lo, hi])
    if rank == 0:
        print(json.dumps({"plumbing": True, "metric": METRIC, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "scaling": args.scaling, "shards": shards,
                          "wall_max_s": wall_max, "global_blocks": global_blocks}), flush=True)
    if group.dist is not None:
        group.dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=16, help="cities per block (config 3: 16)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: one fixed instance of --global-blocks blocks split over the ranks (the "
                         "reference's axis); weak: --blocks-per-gpu blocks per rank")
    ap.add_argument("--global-blocks", type=int, default=65536, help="strong scaling: ./tsp n G instance")
    ap.add_argument("--blocks-per-gpu", type=int, default=16384, help="weak scaling (and the weak probe)")
    ap.add_argument("--k2-n", type=int, default=32, help="cities of the K2 strong-scaling instance")
    ap.add_argument("--k2-seed", type=int, default=35)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-tto", action="store_true", help="skip the time-to-optimal probes")
    ap.add_argument("--no-k2", action="store_true", help="skip the K2 search probes")
    ap.add_argument("--no-k3", action="store_true", help="skip the K3 merge-dominated CLI runs")
    ap.add_argument("--no-ref-multiblock", action="store_true",
                    help="skip the reference-vs-drop-in `./tsp 16 8` runs at P = 1/2/4/8")
    ap.add_argument("--plumbing", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child-k2", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args)
    if args.pmc_child_k2:
        return pmc_child_k2()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing:
        return plumbing(args, world, rank)
    group = Group(world)

    n = args.n
    ndev = max(1, tspgpu.device_count())
    device = local_rank % ndev
    ctx = tspgpu.Context(device=device, strict=False)
    cu, devname = ctx.device_info()
    if args.scaling == "strong":
        global_blocks = args.global_blocks
        lo, hi = strong_bounds(rank, world, global_blocks)
    else:
        global_blocks = args.blocks_per_gpu * world
        lo, hi = shard_bounds(rank, world, args.blocks_per_gpu)
    Bp = hi - lo  # this rank's blocks
    shard = Shard(n, global_blocks, lo, hi)
    d = shard.distances()
    dd, dc, dt = ctx.upload(d), ctx.alloc(max(Bp, 1) * 8), ctx.alloc(max(Bp, 1) * (n + 1) * 4)
    stream = ctx.stream

    ev = {}

    def step():
        ctx.solve_device(dd, n, Bp, dc, dt, stream)

    # the forward / backtracking kernels' own times come from the timed
    # launches themselves: HIP events before, between and after the two
    # kernels of every chunk (variants 5/6; summed by libtspgpu, read after)
    def begin():
        ctx.k1_split_timing(True)
        ctx.timer_start()

    def stop_events():
        ev["ms"] = ctx.timer_stop()  # HIP events on the kernel's stream

    wall_max, _ = timed_steps(step, ctx.synchronize, group, args.warmup, args.steps, begin=begin,
                              end=stop_events)
    kernel_ms = ev["ms"] / args.steps
    variant = ctx.last_variant()
    kname = kernel_name(variant)
    split = None
    if variant in (5, 6):
        f_ms, b_ms = ctx.k1_last_split_ms()
        split = {"forward_kernel_ms": f_ms / args.steps, "backtrack_kernel_ms": b_ms / args.steps,
                 "forward_kernel": kname, "backtrack_kernel": "hk_tiled_backtrack",
                 "source": f"HIP events around both kernels of every chunk of the {args.steps} timed steps "
                           f"(per-step sums)"}
    ctx.k1_split_timing(False)

    # correctness of what was timed: every tour is a permutation whose left fold equals its cost
    cost = ctx.download(dc, (Bp,), np.float64)
    tour = ctx.download(dt, (Bp, n + 1), np.int32)
    for b in range(0, Bp, max(1, Bp // 64)):
        assert sorted(tour[b, :n].tolist()) == list(range(n)) and tour[b, 0] == 0 and tour[b, n] == 0
        acc = 0.0
        for i in range(n):
            acc = acc + d[b, tour[b, i], tour[b, i + 1]]
        assert acc == cost[b], "timed result failed the left-fold check"

    relax = tspgpu.relaxations_per_block(n)
    total_blocks = global_blocks * args.steps
    value = total_blocks * relax / wall_max

    # the other scaling form beside the headline: with strong scaling, every
    # rank also solves a fixed --blocks-per-gpu shard (weak), and vice versa
    other_scaling = None
    if os.environ.get("BENCH_OTHER_SCALING", "1") != "0":
        try:
            other_scaling = scaling_probe(ctx, args, world, rank, group, n, relax)
        except Exception as e:  # noqa: BLE001 - the probe must never cost the headline line
            other_scaling = {"error": f"{type(e).__name__}: {e}"}

    # time to optimal: one block through the ABI (in process), and the whole
    # program as a child process (the reference's definition)
    tto = {}
    if not args.no_tto:
        t_one = []
        one = [shard.block(0)]
        for _ in range(10):
            t = time.perf_counter()
            ctx.solve_cities(one)
            t_one.append((time.perf_counter() - t) * 1e3)
        d1, c1, t1 = ctx.upload(d[:1]), ctx.alloc(8), ctx.alloc((n + 1) * 4)
        ctx.timer_start()
        for _ in range(10):
            ctx.solve_device(d1, n, 1, c1, t1, stream)
        tto["one_block_kernel_ms"] = ctx.timer_stop() / 10
        wide = [ctx.solve_instance(d[0]) for _ in range(5)]
        assert all(w[0] == cost[0] for w in wide), "K1-wide disagrees with K1"
        tto["one_block_whole_gpu_kernel_ms"] = min(w[2] for w in wide)
        tto["one_block_in_process_ms"] = statistics.median(t_one)
        if rank == 0:
            tto["cli_wall_ms"] = {f"n{m}": cli_wall(m) for m in (14, 16)}

    # extension probe: the same launch on the rounded integer matrices (K1 i32)
    i32 = None
    if os.environ.get("BENCH_I32", "1") != "0":
        try:
            di = np.rint(d).astype(np.int32)
            pi, ci, ti = ctx.upload(di), ctx.alloc(Bp * 4), ctx.alloc(Bp * (n + 1) * 4)
            ctx.solve_device_i32(pi, n, Bp, ci, ti, stream)
            ctx.k1_split_timing(True)
            ctx.timer_start()
            for _ in range(5):
                ctx.solve_device_i32(pi, n, Bp, ci, ti, stream)
            i32_ms = ctx.timer_stop() / 5
            i32_split = None
            if ctx.last_variant() in (5, 6):
                f_ms, b_ms = ctx.k1_last_split_ms()
                i32_split = (f_ms / 5, b_ms / 5)
            ctx.k1_split_timing(False)
            ci_h = ctx.download(ci, (Bp,), np.int32)
            ti_h = ctx.download(ti, (Bp, n + 1), np.int32)
            for b in range(0, Bp, max(1, Bp // 64)):
                assert sum(int(di[b, ti_h[b, i], ti_h[b, i + 1]]) for i in range(n)) == int(ci_h[b])
            for p_ in (pi, ci, ti):
                ctx.free(p_)
            i32 = {"kernel_ms_per_launch": i32_ms, "blocks_per_s": Bp / (i32_ms * 1e-3),
                   "relaxations_per_s": Bp * relax / (i32_ms * 1e-3), "variant": ctx.last_variant(),
                   "note": "extension (no reference counterpart): rint(distances) as int32, same DP and tie rule"}
            if i32_split:
                i32.update(forward_kernel_ms=i32_split[0], backtrack_kernel_ms=i32_split[1],
                           forward_relaxations_per_s=Bp * relax / (i32_split[0] * 1e-3))
        except Exception as e:  # noqa: BLE001 - the probe must never cost the headline line
            i32 = {"error": f"{type(e).__name__}: {e}"}

    k2 = k2s = exh = tsplib = None
    if not args.no_k2 and os.environ.get("BENCH_K2", "1") != "0":
        try:
            kgroup, backend = k2_group(world, local_rank)
        except Exception as e:  # noqa: BLE001
            kgroup, backend = None, f"error: {e}"
        if rank == 0:
            try:
                exh = k2_exhaustive(ctx)
            except Exception as e:  # noqa: BLE001
                exh = {"error": f"{type(e).__name__}: {e}"}
            try:
                tsplib = config4_tsplib(ctx)
            except Exception as e:  # noqa: BLE001
                tsplib = {"error": f"{type(e).__name__}: {e}"}
        try:
            k2 = k2_single_instance(ctx, n, kgroup, backend, world)
        except Exception as e:  # noqa: BLE001
            k2 = {"error": f"{type(e).__name__}: {e}"}
        try:
            k2s = k2_strong_scaling(ctx, args.k2_n, args.k2_seed, kgroup, backend, world, rank)
            walls = group.gather(k2s["rank_wall_ms"])
            # every rank's host/device split (its wall by host phase, its kernels)
            k2s["rank_split"] = group.gather({"rank": rank, "wall_ms": k2s["rank_wall_ms"],
                                              "kernel_ms": k2s["rank_kernel_ms"],
                                              "host_phases_ms": k2s.get("host_phases_ms")})
            k2s["time_to_optimal_ms"] = max(walls)
            k2s["bb_nodes_per_s"] = k2s["bb_nodes_expanded"] / (k2s["time_to_optimal_ms"] * 1e-3)
            k2s["rank_walls_ms"] = walls
        except Exception as e:  # noqa: BLE001
            k2s = {"error": f"{type(e).__name__}: {e}"}

    if rank != 0:
        if group.dist is not None:
            group.barrier()
        return
    alg_bytes_per_block = tspgpu.table_bytes_per_block(n)
    prof = None
    if world == 1 and not args.no_pmc:
        prof = pmc_profile(n, min(Bp, 4096), cu, kname)
    peaks = valu_peaks() if world == 1 else None
    if i32 and "relaxations_per_s" in i32 and (peaks or {}).get("i32 relaxation min-only (add,min)"):
        # K1 on int32 distances against the integer VALU issue rate of its own
        # min-only relaxation (v_add_u32 + v_min_i32, registers only, this GPU),
        # the forward kernel's time as for the f64 headline
        pk = peaks["i32 relaxation min-only (add,min)"]
        ach = i32.get("forward_relaxations_per_s", i32["relaxations_per_s"])
        spec = VALU_SPEC_I32 / 2  # 2 lane-instructions (v_add_u32, v_min_i32) per relaxation
        i32["valu_roofline"] = {"bound": "valu (int32)", "achieved_relax_per_s": ach, "peak_relax_per_s": spec,
                                "frac": ach / spec, "peak_source": "spec: 78.6 T int32 lane-instructions/s / 2",
                                "measured_peak_relax_per_s": pk, "frac_of_measured_peak": ach / pk,
                                "note": "forward kernel alone (HIP events around it in each chunk), like the f64 line; "
                                        "measured peak = bin/ubench's add+min mix on this GPU"}
    dom_ms = split["forward_kernel_ms"] if split else kernel_ms  # the dominant kernel's own time
    relax_s_kernel = Bp * relax / (dom_ms * 1e-3)
    roof = roofline(variant, kname, n, Bp, dom_ms, relax_s_kernel, alg_bytes_per_block, prof, peaks)
    if world == 1 and not args.no_pmc and k2 and "bb_nodes_expanded" in k2:
        try:
            k2["pmc"] = k2_pmc(cu, peaks, k2["bb_nodes_expanded"], k2["kernel_ms"])
        except Exception as e:  # noqa: BLE001
            k2["pmc"] = {"error": f"{type(e).__name__}: {e}"}
    cpu = cpu_opt = refmb = k3 = None
    if world == 1 and not args.no_k3:
        try:
            k3 = k3_merge()
        except Exception as e:  # noqa: BLE001
            k3 = {"error": f"{type(e).__name__}: {e}"}
    if world == 1 and not args.no_ref_multiblock:
        try:
            refmb = reference_multiblock(n)
        except Exception as e:  # noqa: BLE001
            refmb = {"error": f"{type(e).__name__}: {e}"}
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(n)
        try:
            cpu_opt = cpu_optimized(n)
        except Exception as e:  # noqa: BLE001
            cpu_opt = {"error": f"{type(e).__name__}: {e}"}
    # both halves of the metric, first class (the headline `value` is K1's
    # relaxations/s; the B&B search's nodes/s and time to the optimal tour
    # of the 16-city instance are K2's)
    headline = {
        "k1_dp_relaxations_per_s": value,
        "k1_roofline_frac": (roof or {}).get("frac"),
        "k2_search_nodes_per_s": (k2 or {}).get("bb_nodes_per_s"),
        "k2_time_to_optimal_ms_in_process": (k2 or {}).get("time_to_optimal_ms"),
        "k2_kernel_ms": (k2 or {}).get("kernel_ms"),
        "k2_instance": (k2 or {}).get("instance"),
        "time_to_optimal_ms_program": ((tto or {}).get("cli_wall_ms") or {}).get("n16", {}).get("program_ms")
        if isinstance(((tto or {}).get("cli_wall_ms") or {}).get("n16"), dict) else None,
        "time_to_optimal_ms_program_after_runtime_startup":
        ((tto or {}).get("cli_wall_ms") or {}).get("n16", {}).get("program_ms_after_runtime_startup")
        if isinstance(((tto or {}).get("cli_wall_ms") or {}).get("n16"), dict) else None,
        "k2_strong_scaling_time_to_optimal_ms": (k2s or {}).get("time_to_optimal_ms"),
        "k2_strong_scaling_nodes_per_s": (k2s or {}).get("bb_nodes_per_s"),
    }
    line = {
        "metric": METRIC,
        "value": value,
        "unit": UNIT,
        "headline": headline,
        # GPUs actually used: ranks sharing a device (a rehearsal on a smaller
        # box) do not add GPUs, and the line says so
        "n_gpus": min(world, ndev),
        "ranks": world,
        "ranks_per_gpu": -(-world // ndev),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: the reference's own generator (srand(0), ./tsp n B 1000 1000), no dataset",
        "config": {"workload": f"{n}-city blocks, exact Held-Karp per block (config 3 cities/block; "
                               f"./tsp {n} {global_blocks} 1000 1000 instance)",
                   "n": n, "blocks_rank0": Bp, "global_blocks": global_blocks,
                   "parallelism": f"{args.scaling} scaling: blocks sharded contiguously over {world} rank(s) "
                                  f"(one per GPU; the reference's per-rank counts), no data-path collective",
                   "k1_variant": variant, "kernel": kname},
        "blocks_per_s": total_blocks / wall_max,
        "kernel_ms_per_launch": kernel_ms,
        "k1_kernel_split": split,
        "other_scaling": other_scaling,
        "reference_multiblock": refmb,
        "time_to_optimal": tto,
        "roofline": roof,
        "counters": prof,
        "valu_peaks_measured": peaks,
        "cpu_baseline": cpu,
        "cpu_optimized": cpu_opt,
        "k2_single_instance": k2,
        "k2_strong_scaling": k2s,
        "k2_exhaustive_14": exh,
        "k3_merge": k3,
        "config4_tsplib": tsplib,
        "k1_i32_extension": i32,
        "device": devname,
        "cus": cu,
    }
    print(json.dumps(line), flush=True)
    if group.dist is not None:
        group.barrier()


def roofline(variant, kname, n, Bp, kernel_ms, relax_s, alg_bytes_per_block, prof, peaks):
    """The dominant kernel against the ceiling that binds it.

    VALU: a DP relaxation needs at least two VALU instructions (v_add_f64,
    v_min_f64; the argmin that gives the tour is kept only for the top rows in
    variant 5 and recomputed on the path by the backtracking kernel); the peak
    is that min-only mix's issue rate measured on this GPU (bin/ubench), so
    frac = relaxations/s of the forward kernel / peak relaxations/s.  For the
    other variants (argmin in every relaxation) the 4-instruction mix is the
    reference.
    Memory: the bytes that left L2 toward memory per launch (PMC), against
    8 TB/s (an upper bound on HBM: Infinity-Cache hits are included).
    The line reports whichever fraction is higher as `roofline` (the binding
    one) and the other as `other`."""
    mix, per = (("f64 relaxation min-only (add,min)", 2) if variant in (5, 6)
                else ("f64 relaxation+argmin (add,cmp,cndmask,min)", 4))
    peak_relax = (peaks or {}).get(mix)
    scale = Bp / (prof or {}).get("blocks_per_launch", Bp)
    hbm = (prof or {}).get("hbm_bytes")
    hbm = hbm * scale if hbm is not None else None
    fabric = None
    if prof and "fabric_read_bytes" in prof:
        fabric = (prof["fabric_read_bytes"] + prof["fabric_write_bytes"]) * scale
    # the f64 VALU spec (MI355X_MICROARCH.md: half the f32 vector rate) is the
    # peak; the same mix measured by bin/ubench on this GPU rides along
    spec_relax = VALU_SPEC_F64 / per
    valu = {"bound": "valu", "achieved": per * relax_s / 1e12, "peak": VALU_SPEC_F64 / 1e12,
            "unit": "T VALU lane-instructions/s", "frac": relax_s / spec_relax, "traffic": hbm,
            "peak_source": "spec: 256 CU x 4 SIMD x 16 f64 lanes/clk x 2.4 GHz",
            "measured_peak": per * peak_relax / 1e12 if peak_relax else None,
            "frac_of_measured_peak": relax_s / peak_relax if peak_relax else None,
            "note": f"{kname} (n={n}): {per} VALU instructions per DP relaxation ({mix}) x {Bp} blocks x "
                    f"{tspgpu.relaxations_per_block(n):.0f} relaxations / the kernel's own HIP-event time "
                    f"({kernel_ms:.3f} ms); measured_peak = the same mix by bin/ubench on this GPU; "
                    f"traffic = memory-side bytes per launch (PMC)"}
    mem = None
    if hbm is not None:
        mem = {"bound": "hbm (upper bound: Infinity-Cache hits included)", "achieved": hbm / (kernel_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
               "frac": hbm / (kernel_ms * 1e-3) / HBM_PEAK, "traffic": hbm,
               "note": f"memory-side bytes per launch = PMC FETCH_SIZE x2 + WRITE_SIZE ({fabric:.4g}; calibrated on 8-B "
                       f"loads/stores; Infinity-Cache hits are counted too, TCC_EA0_*_DRAM does not split them), vs the "
                       f"HBM peak; the layer-by-layer algorithmic table bytes would be {alg_bytes_per_block * Bp:.4g}"}
    if valu and mem:
        # The memory view counts every byte that left L2 toward memory (the
        # gfx950 counters cannot separate Infinity-Cache hits from HBM reads:
        # profiles/r02/pmc_calibration_dram_counters.txt), so it is an upper
        # bound on HBM traffic; the kernel is priced against the VALU issue
        # rate of its own instruction mix unless memory is clearly the wall.
        a, b = (mem, valu) if mem["frac"] > max(0.6, valu["frac"]) else (valu, mem)
        return dict(a, other=b)
    return valu or mem or {"bound": "unknown", "achieved": None, "peak": None, "unit": None, "frac": None,
                           "traffic": None, "note": "no PMC / ubench data in this run"}


if __name__ == "__main__":
    main()
