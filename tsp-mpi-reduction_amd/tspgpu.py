"""ctypes binding of libtspgpu (include/tspgpu.h) for tests and bench.py.

This is the same C ABI a ctypes user of the reference's block solver would
bind.  It never falls back to CPU code: if lib/libtspgpu.so
is missing or no HIP device is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import errno
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# TSPGPU_LIB: another build of the same ABI (development A/B experiments)
LIB_PATH = os.environ.get("TSPGPU_LIB") or os.path.join(PKG_DIR, "lib", "libtspgpu.so")
HOST_LIB_PATH = os.path.join(PKG_DIR, "lib", "libtsphost.so")
TSP_BIN = os.path.join(PKG_DIR, "bin", "tsp")

EXPORTED_SYMBOLS = (
    "tspgpu_version", "tspgpu_strerror", "tspgpu_tour_length", "tspgpu_distance_matrix", "tspgpu_validate",
    "tspgpu_ctx_create", "tspgpu_ctx_destroy", "tspgpu_solve_blocks", "tspgpu_solve_cities",
    "tspgpu_solve_blocks_device", "tspgpu_solve", "tspgpu_last_grid", "tspgpu_relaxations_per_block",
    "tspgpu_table_bytes_per_block", "tspgpu_device_alloc", "tspgpu_device_free", "tspgpu_memcpy_htod",
    "tspgpu_memcpy_dtoh", "tspgpu_stream", "tspgpu_synchronize", "tspgpu_timer_start", "tspgpu_timer_stop",
    "tspgpu_device_info", "tspgpu_last_variant", "tspgpu_k1_split_timing", "tspgpu_k1_last_split_ms", "tspgpu_device_count", "tspgpu_stream_create",
    "tspgpu_stream_destroy", "tspgpu_stream_synchronize",
    # K2
    "tspgpu_search_solve", "tspgpu_search_enumerate", "tspgpu_search_create", "tspgpu_search_create_ex",
    "tspgpu_search_destroy", "tspgpu_search_info",
    "tspgpu_search_set_bound", "tspgpu_search_start", "tspgpu_search_step", "tspgpu_search_run_all",
    "tspgpu_search_timing", "tspgpu_search_incumbent_device", "tspgpu_search_chain", "tspgpu_search_tie_slot",
    "tspgpu_search_counters", "tspgpu_search_reset_records", "tspgpu_search_records", "tspgpu_heuristic_tour",
    "tspgpu_heuristic_tour_starts",
    "tspgpu_select_tour", "tspgpu_tie_tour", "tspgpu_tie_tour_gpu", "tspgpu_tie_tour_records", "tspgpu_tie_key",
    # K3
    "tspgpu_merge", "tspgpu_reduce",
    # K1-wide
    "tspgpu_solve_instance",
    # K1 on integer distances
    "tspgpu_validate_i32", "tspgpu_solve_blocks_i32", "tspgpu_solve_blocks_i32_device",
    # tuning / test knobs
    "tspgpu_tuning_set", "tspgpu_tuning_clear",
)

F64, I32 = 0, 1
SEARCH_MAX_CITIES = 32
MAX_CITIES = 20  # TSPGPU_MAX_CITIES: the batched K1 (extension sizes above the reference's 16)


class TourRecord(ctypes.Structure):
    """tspgpu_tour_record: cost bits + inner cities t1..tN."""
    _fields_ = [("cost", ctypes.c_uint64), ("city", ctypes.c_uint8 * 32)]


class SearchStats(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_uint64), ("records", ctypes.c_uint64), ("optimal_tours", ctypes.c_uint64),
                ("items", ctypes.c_uint64), ("depth", ctypes.c_int), ("phases", ctypes.c_int),
                ("fallback", ctypes.c_int), ("rounds", ctypes.c_int), ("kernel_ms", ctypes.c_double),
                ("lane_steps", ctypes.c_uint64), ("active_steps", ctypes.c_uint64), ("item_loads", ctypes.c_uint64),
                ("tie", ctypes.c_int), ("tie_checked", ctypes.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class TieSlot(ctypes.Structure):
    """tspgpu_tie_slot: a shard's least tie key at one cost."""
    _fields_ = [("w0", ctypes.c_uint64), ("w1", ctypes.c_uint64), ("found", ctypes.c_int),
                ("overflow", ctypes.c_int)]


LEVEL_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


class City(ctypes.Structure):
    """tspgpu_city == the reference's City (assignment2.h:13-18)."""
    _fields_ = [("id", ctypes.c_int32), ("x", ctypes.c_double), ("y", ctypes.c_double)]


class Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("strict", ctypes.c_int), ("slots", ctypes.c_int),
                ("reserved", ctypes.c_int * 5)]


class TspGpuError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {lib().tspgpu_strerror(code).decode()} ({code})")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not built (make -C tsp-mpi-reduction_amd)")
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        vp = ctypes.c_void_p
        L.tspgpu_version.restype = ctypes.c_int
        L.tspgpu_strerror.argtypes = [ctypes.c_int]
        L.tspgpu_strerror.restype = ctypes.c_char_p
        L.tspgpu_tour_length.argtypes = [ctypes.c_int]
        L.tspgpu_distance_matrix.argtypes = [ctypes.POINTER(City), ctypes.c_int, ctypes.c_int, dp]
        L.tspgpu_validate.argtypes = [dp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.tspgpu_ctx_create.argtypes = [ctypes.POINTER(Opts), ctypes.POINTER(vp)]
        L.tspgpu_ctx_destroy.argtypes = [vp]
        L.tspgpu_solve_blocks.argtypes = [vp, dp, ctypes.c_int, ctypes.c_int, dp, ip]
        L.tspgpu_solve_cities.argtypes = [vp, ctypes.POINTER(City), ctypes.c_int, ctypes.c_int, dp, ip]
        L.tspgpu_solve_blocks_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.tspgpu_validate_i32.argtypes = [ip, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.tspgpu_solve_blocks_i32.argtypes = [vp, ip, ctypes.c_int, ctypes.c_int, ip, ip]
        L.tspgpu_solve_blocks_i32_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.tspgpu_solve.argtypes = [dp, ctypes.c_int, ctypes.c_int, dp, ip, ctypes.POINTER(Opts)]
        L.tspgpu_last_grid.argtypes = [vp]
        L.tspgpu_last_variant.argtypes = [vp]
        L.tspgpu_k1_split_timing.argtypes = [vp, ctypes.c_int]
        L.tspgpu_k1_last_split_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        L.tspgpu_device_count.argtypes = []
        L.tspgpu_relaxations_per_block.argtypes = [ctypes.c_int]
        L.tspgpu_relaxations_per_block.restype = ctypes.c_double
        L.tspgpu_table_bytes_per_block.argtypes = [ctypes.c_int]
        L.tspgpu_table_bytes_per_block.restype = ctypes.c_double
        L.tspgpu_device_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
        L.tspgpu_device_free.argtypes = [vp, vp]
        L.tspgpu_memcpy_htod.argtypes = [vp, vp, vp, ctypes.c_size_t]
        L.tspgpu_memcpy_dtoh.argtypes = [vp, vp, vp, ctypes.c_size_t]
        L.tspgpu_stream.argtypes = [vp]
        L.tspgpu_stream.restype = vp
        L.tspgpu_synchronize.argtypes = [vp]
        L.tspgpu_stream_create.argtypes = [vp, ctypes.POINTER(vp)]
        L.tspgpu_stream_destroy.argtypes = [vp, vp]
        L.tspgpu_stream_synchronize.argtypes = [vp, vp]
        L.tspgpu_timer_start.argtypes = [vp]
        L.tspgpu_timer_stop.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
        L.tspgpu_device_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.tspgpu_search_solve.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, dp, ip, ctypes.POINTER(SearchStats)]
        L.tspgpu_search_enumerate.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, dp, ip, ctypes.POINTER(SearchStats)]
        L.tspgpu_search_create.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.POINTER(vp)]
        L.tspgpu_search_create_ex.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp)]
        L.tspgpu_search_destroy.argtypes = [vp]
        L.tspgpu_search_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), u64p, u64p]
        L.tspgpu_search_set_bound.argtypes = [vp, ctypes.c_double]
        L.tspgpu_search_start.argtypes = [vp]
        L.tspgpu_search_step.argtypes = [vp, u64p]
        L.tspgpu_search_run_all.argtypes = [vp]
        L.tspgpu_search_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        L.tspgpu_search_incumbent_device.argtypes = [vp]
        L.tspgpu_search_incumbent_device.restype = vp
        L.tspgpu_search_counters.argtypes = [vp, u64p, u64p, u64p]
        L.tspgpu_search_chain.argtypes = [vp, ctypes.c_int, LEVEL_HOOK, vp, ctypes.POINTER(ctypes.c_int)]
        L.tspgpu_search_tie_slot.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(TieSlot)]
        L.tspgpu_search_reset_records.argtypes = [vp, ctypes.c_uint]
        L.tspgpu_search_records.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(TourRecord), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]
        L.tspgpu_heuristic_tour.argtypes = [vp, ctypes.c_int, ctypes.c_int, dp, ip]
        L.tspgpu_heuristic_tour_starts.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, ip]
        L.tspgpu_select_tour.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(TourRecord), ctypes.c_int,
                                         ctypes.c_uint64, ip]
        L.tspgpu_tie_tour.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ip]
        L.tspgpu_tuning_set.argtypes = [ctypes.c_char_p, ctypes.c_double]
        L.tspgpu_tuning_clear.argtypes = [ctypes.c_char_p]
        L.tspgpu_tie_tour_gpu.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint64, ip]
        L.tspgpu_tie_tour_records.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.POINTER(TourRecord), ctypes.c_int, ip]
        L.tspgpu_tie_key.argtypes = [ctypes.c_int, ip, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        cp = ctypes.POINTER(City)
        L.tspgpu_solve_instance.argtypes = [vp, dp, ctypes.c_int, dp, ip, dp]
        L.tspgpu_merge.argtypes = [vp, cp, ctypes.c_int, ctypes.c_double, cp, ctypes.c_int, ctypes.c_double, cp, dp]
        L.tspgpu_reduce.argtypes = [vp, cp, ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, dp, ctypes.c_char_p,
                                    ctypes.c_int]
        _lib = L
    return _lib


def tune(name: str, value) -> None:
    """Set a tuning / test knob (tspgpu_tuning_set; include/tspgpu.h
    "Tuning"): process-wide, read where the knob is used (K1 knobs at
    Context creation, K2 knobs at search creation)."""
    rc = lib().tspgpu_tuning_set(name.encode(), float(value))
    if rc:
        raise TspGpuError(rc, f"tspgpu_tuning_set({name})")


def tune_from_environ() -> None:
    """Development tools only (tools/*.py): every TSPGPU_<KNOB>=value of this
    process's environment as tune(KNOB, value).  The library itself reads no
    environment variable; neither the tests nor bench.py call this."""
    for k, v in os.environ.items():
        if k.startswith("TSPGPU_") and k != "TSPGPU_LIB":
            tune(k[len("TSPGPU_"):], float(v))


def untune(name: str | None = None) -> None:
    """Back to the default (None: every knob)."""
    rc = lib().tspgpu_tuning_clear(name.encode() if name else None)
    if rc:
        raise TspGpuError(rc, f"tspgpu_tuning_clear({name})")


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def device_count() -> int:
    """Visible HIP devices (initialises HIP in this process)."""
    return lib().tspgpu_device_count()


def tour_length(n: int) -> int:
    return lib().tspgpu_tour_length(n)


def relaxations_per_block(n: int) -> float:
    return lib().tspgpu_relaxations_per_block(n)


def table_bytes_per_block(n: int) -> float:
    return lib().tspgpu_table_bytes_per_block(n)


def cities_array(blocks):
    """blocks: list of blocks, each a list of (id, x, y) -> (ctypes City array, n, B)."""
    B = len(blocks)
    n = len(blocks[0]) if B else 0
    arr = (City * max(1, B * n))()
    for b, blk in enumerate(blocks):
        assert len(blk) == n
        for j, (cid, x, y) in enumerate(blk):
            c = arr[b * n + j]
            c.id, c.x, c.y = int(cid), float(x), float(y)
    return arr, n, B


def distance_matrix(blocks) -> np.ndarray:
    """Host libm distances, bit-exact with computeDistanceMatrix (assignment2.h:184-200)."""
    arr, n, B = cities_array(blocks)
    d = np.zeros((B, n, n), dtype=np.float64)
    rc = lib().tspgpu_distance_matrix(arr, n, B, _dp(d))
    if rc:
        raise TspGpuError(rc, "tspgpu_distance_matrix")
    return d


def distance_matrix_array(arr, n: int, B: int) -> np.ndarray:
    """Same, from a ctypes City array of B*n cities."""
    d = np.zeros((B, n, n), dtype=np.float64)
    rc = lib().tspgpu_distance_matrix(arr, n, B, _dp(d))
    if rc:
        raise TspGpuError(rc, "tspgpu_distance_matrix")
    return d


def validate(dist: np.ndarray, strict: bool = False) -> int:
    dist = np.ascontiguousarray(dist, dtype=np.float64)
    B, n, _ = dist.shape
    return lib().tspgpu_validate(_dp(dist), n, B, int(strict))


def validate_i32(dist: np.ndarray, strict: bool = False) -> int:
    dist = np.ascontiguousarray(dist, dtype=np.int32)
    B, n, _ = dist.shape
    return lib().tspgpu_validate_i32(_ip(dist), n, B, int(strict))


class Context:
    """Owns a tspgpu_ctx (device memory, stream) on one HIP device."""

    def __init__(self, device: int = -1, strict: bool = False, slots: int = 0):
        o = Opts(device, int(strict), slots)
        h = ctypes.c_void_p()
        rc = lib().tspgpu_ctx_create(ctypes.byref(o), ctypes.byref(h))
        if rc:
            raise TspGpuError(rc, "tspgpu_ctx_create")
        self.handle = h

    def close(self):
        # (destroy order is free in the C ABI: live searches keep the
        # context, the last Search.close releases it — include/tspgpu.h)
        if self.handle:
            lib().tspgpu_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def solve_blocks(self, dist: np.ndarray):
        """dist: (B, n, n) float64 -> (costs (B,), tours (B, n+1) int32, -1 padded)."""
        dist = np.ascontiguousarray(dist, dtype=np.float64)
        B, n, _ = dist.shape
        cost = np.zeros(B, dtype=np.float64)
        tour = np.full((B, n + 1), -1, dtype=np.int32)
        rc = lib().tspgpu_solve_blocks(self.handle, _dp(dist), n, B, _dp(cost), _ip(tour))
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_blocks")
        return cost, tour

    def solve_blocks_i32(self, dist: np.ndarray):
        """dist: (B, n, n) int32 -> (costs (B,) int32, tours (B, n+1) int32, -1 padded)."""
        dist = np.ascontiguousarray(dist, dtype=np.int32)
        B, n, _ = dist.shape
        cost = np.zeros(B, dtype=np.int32)
        tour = np.full((B, n + 1), -1, dtype=np.int32)
        rc = lib().tspgpu_solve_blocks_i32(self.handle, _ip(dist), n, B, _ip(cost), _ip(tour))
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_blocks_i32")
        return cost, tour

    def solve_device_i32(self, d_dist_ptr: int, n: int, nblocks: int, d_cost_ptr: int, d_tour_ptr: int,
                         stream_ptr: int = 0):
        rc = lib().tspgpu_solve_blocks_i32_device(self.handle, d_dist_ptr, n, nblocks, d_cost_ptr, d_tour_ptr,
                                                  stream_ptr)
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_blocks_i32_device")

    def solve_cities(self, blocks):
        arr, n, B = cities_array(blocks)
        cost = np.zeros(B, dtype=np.float64)
        tour = np.full((B, n + 1), -1, dtype=np.int32)
        rc = lib().tspgpu_solve_cities(self.handle, arr, n, B, _dp(cost), _ip(tour))
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_cities")
        return cost, tour

    def solve_device(self, d_dist_ptr: int, n: int, nblocks: int, d_cost_ptr: int, d_tour_ptr: int,
                     stream_ptr: int = 0):
        rc = lib().tspgpu_solve_blocks_device(self.handle, d_dist_ptr, n, nblocks, d_cost_ptr, d_tour_ptr,
                                              stream_ptr)
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_blocks_device")

    def last_grid(self) -> int:
        return lib().tspgpu_last_grid(self.handle)

    def last_variant(self) -> int:
        """K1 variant of the last batched launch (6: hk_sub_kernel, 5: hk_tiled_kernel, else heldkarp_kernel)."""
        return lib().tspgpu_last_variant(self.handle)

    def k1_split_timing(self, enable: bool = True):
        """Record an event between variant 5's forward and backtracking kernels."""
        self._check(lib().tspgpu_k1_split_timing(self.handle, int(enable)), "tspgpu_k1_split_timing")

    def k1_last_split_ms(self):
        """(forward_ms, backtrack_ms) of the last variant-5 launch (waits for it)."""
        f, b = ctypes.c_float(), ctypes.c_float()
        self._check(lib().tspgpu_k1_last_split_ms(self.handle, ctypes.byref(f), ctypes.byref(b)),
                    "tspgpu_k1_last_split_ms")
        return f.value, b.value

    def _check(self, rc, what):
        if rc:
            raise TspGpuError(rc, what)

    def alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        self._check(lib().tspgpu_device_alloc(self.handle, nbytes, ctypes.byref(p)), "tspgpu_device_alloc")
        return p.value

    def free(self, ptr: int):
        self._check(lib().tspgpu_device_free(self.handle, ptr), "tspgpu_device_free")

    def upload(self, arr: np.ndarray) -> int:
        arr = np.ascontiguousarray(arr)
        p = self.alloc(arr.nbytes)
        self._check(lib().tspgpu_memcpy_htod(self.handle, p, arr.ctypes.data, arr.nbytes), "tspgpu_memcpy_htod")
        return p

    def download(self, ptr: int, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        self._check(lib().tspgpu_memcpy_dtoh(self.handle, out.ctypes.data, ptr, out.nbytes), "tspgpu_memcpy_dtoh")
        return out

    @property
    def stream(self) -> int:
        return lib().tspgpu_stream(self.handle) or 0

    def synchronize(self, stream: int | None = None):
        if stream is None:
            self._check(lib().tspgpu_synchronize(self.handle), "tspgpu_synchronize")
        else:
            self._check(lib().tspgpu_stream_synchronize(self.handle, stream), "tspgpu_stream_synchronize")

    def stream_create(self) -> int:
        s = ctypes.c_void_p()
        self._check(lib().tspgpu_stream_create(self.handle, ctypes.byref(s)), "tspgpu_stream_create")
        return s.value

    def stream_destroy(self, stream: int):
        self._check(lib().tspgpu_stream_destroy(self.handle, stream), "tspgpu_stream_destroy")

    def timer_start(self):
        self._check(lib().tspgpu_timer_start(self.handle), "tspgpu_timer_start")

    def timer_stop(self) -> float:
        ms = ctypes.c_float()
        self._check(lib().tspgpu_timer_stop(self.handle, ctypes.byref(ms)), "tspgpu_timer_stop")
        return ms.value

    def solve_instance(self, dist):
        """K1-wide: one instance over the whole GPU -> (cost, tour (n+1,), kernel ms)."""
        d = np.ascontiguousarray(dist, dtype=np.float64)
        n = d.shape[0]
        cost, ms = ctypes.c_double(), ctypes.c_double()
        tour = np.zeros(n + 1, dtype=np.int32)
        rc = lib().tspgpu_solve_instance(self.handle, _dp(d), n, ctypes.byref(cost), _ip(tour), ctypes.byref(ms))
        if rc:
            raise TspGpuError(rc, "tspgpu_solve_instance")
        return cost.value, tour, ms.value

    def merge(self, p1, c1, p2, c2):
        """K3 mergeBlocks: paths are lists of (id, x, y) -> (merged path, cost)."""
        a1, _, _ = cities_array([p1])
        a2, _, _ = cities_array([p2])
        out = (City * (len(p1) + len(p2)))()
        cost = ctypes.c_double()
        rc = lib().tspgpu_merge(self.handle, a1, len(p1), c1, a2, len(p2), c2, out, ctypes.byref(cost))
        if rc < 0:
            raise TspGpuError(rc, "tspgpu_merge")
        return [(out[i].id, out[i].x, out[i].y) for i in range(rc)], cost.value

    def reduce(self, paths, costs, nprocs: int):
        """K3 reduction: paths (B lists of L cities), costs (B,) -> (final cost, log text)."""
        B, L = len(paths), len(paths[0])
        flat, _, _ = cities_array(paths)
        c = np.ascontiguousarray(costs, dtype=np.float64)
        final = ctypes.c_double()
        log = ctypes.create_string_buffer(1 << 20)
        rc = lib().tspgpu_reduce(self.handle, flat, L, _dp(c), B, nprocs, ctypes.byref(final), log, len(log))
        if rc:
            raise TspGpuError(rc, "tspgpu_reduce")
        return final.value, log.value.decode()

    def device_info(self):
        cu = ctypes.c_int()
        name = ctypes.create_string_buffer(256)
        self._check(lib().tspgpu_device_info(self.handle, ctypes.byref(cu), name, 256), "tspgpu_device_info")
        return cu.value, name.value.decode()


def _search_dist(dist):
    """(n, n) matrix -> (contiguous array, dtype code): float -> F64, integer -> I32."""
    dist = np.asarray(dist)
    if np.issubdtype(dist.dtype, np.integer):
        return np.ascontiguousarray(dist, dtype=np.int32), I32
    return np.ascontiguousarray(dist, dtype=np.float64), F64


def cost_bits(cost, dtype: int) -> int:
    """The 64-bit incumbent word of a cost (f64 IEEE bits or the integer)."""
    if dtype == F64:
        return int(np.array([cost], dtype=np.float64).view(np.uint64)[0])
    return int(cost)


def bits_cost(bits: int, dtype: int):
    if dtype == F64:
        return float(np.array([bits], dtype=np.uint64).view(np.float64)[0])
    return int(np.uint32(bits).view(np.int32))


def heuristic_tour(dist, first: int = 0, step: int = 1):
    """Multi-start tour (an upper bound): the start cities first, first+step, ...
    -> (cost, tour), or (None, None) when the range holds no start city."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    cost = ctypes.c_double()
    tour = np.zeros(n + 1, dtype=np.int32)
    rc = lib().tspgpu_heuristic_tour_starts(d.ctypes.data, dt, n, first, step, ctypes.byref(cost), _ip(tour))
    if rc == -errno.ENOENT:
        return None, None
    if rc:
        raise TspGpuError(rc, "tspgpu_heuristic_tour_starts")
    return cost.value, tour


def read_tsplib(path):
    """A TSPLIB file -> (name, int32 distance matrix): EDGE_WEIGHT_TYPE EUC_2D,
    CEIL_2D, ATT, GEO (TSPLIB95's integer distance functions; GEO degrees
    truncated like Concorde) or EXPLICIT (FULL_MATRIX, UPPER_ROW, LOWER_ROW,
    UPPER_DIAG_ROW, LOWER_DIAG_ROW).  The same reader as bin/tsp_search --tsplib
    (host/tsp_search.cpp); integer matrices run the exact integer mode."""
    import math

    hdr, coords, weights, section = {}, [], [], None
    for line in open(path):
        t = line.strip()
        if not t or t == "EOF":
            if t == "EOF":
                break
            continue
        if t.startswith("NODE_COORD_SECTION"):
            section = "coord"
            continue
        if t.startswith("EDGE_WEIGHT_SECTION"):
            section = "weight"
            continue
        if t.split()[0].endswith("_SECTION"):
            section = "skip"
            continue
        if section is None and ":" in t:
            k, v = t.split(":", 1)
            hdr[k.strip().upper()] = v.strip()
            continue
        if section == "coord":
            f = t.split()
            coords.append((float(f[1]), float(f[2])))
        elif section == "weight":
            weights.extend(int(float(x)) for x in t.split())
    n = int(hdr["DIMENSION"])
    kind = hdr.get("EDGE_WEIGHT_TYPE", "EUC_2D").upper()
    d = np.zeros((n, n), dtype=np.int64)
    if kind == "EXPLICIT":
        fmt = hdr.get("EDGE_WEIGHT_FORMAT", "FULL_MATRIX").upper()
        it = iter(weights)
        for i in range(n):
            if fmt == "FULL_MATRIX":
                cols = range(n)
            elif fmt == "UPPER_ROW":
                cols = range(i + 1, n)
            elif fmt == "LOWER_ROW":
                cols = range(i)
            elif fmt == "UPPER_DIAG_ROW":
                cols = range(i, n)
            elif fmt == "LOWER_DIAG_ROW":
                cols = range(i + 1)
            else:
                raise ValueError(f"EDGE_WEIGHT_FORMAT {fmt} not supported")
            for j in cols:
                d[i, j] = next(it)
                if fmt != "FULL_MATRIX":
                    d[j, i] = d[i, j]
    else:
        if len(coords) != n:
            raise ValueError("NODE_COORD_SECTION does not hold DIMENSION cities")

        def geo(v):
            deg = float(int(v))
            return 3.141592 * (deg + 5.0 * (v - deg) / 3.0) / 180.0

        for i in range(n):
            for j in range(n):
                if i == j:
                    continue
                (xi, yi), (xj, yj) = coords[i], coords[j]
                if kind == "GEO":
                    q1 = math.cos(geo(yi) - geo(yj))
                    q2 = math.cos(geo(xi) - geo(xj))
                    q3 = math.cos(geo(xi) + geo(xj))
                    d[i, j] = int(6378.388 * math.acos(0.5 * ((1.0 + q1) * q2 - (1.0 - q1) * q3)) + 1.0)
                elif kind == "ATT":
                    r = math.sqrt(((xi - xj) ** 2 + (yi - yj) ** 2) / 10.0)
                    t_ = int(r + 0.5)
                    d[i, j] = t_ + 1 if t_ < r else t_
                elif kind == "CEIL_2D":
                    d[i, j] = int(math.ceil(math.sqrt((xi - xj) ** 2 + (yi - yj) ** 2)))
                elif kind == "EUC_2D":
                    d[i, j] = int(math.sqrt((xi - xj) ** 2 + (yi - yj) ** 2) + 0.5)
                else:
                    raise ValueError(f"EDGE_WEIGHT_TYPE {kind} not supported")
    return hdr.get("NAME", os.path.basename(path)), d.astype(np.int32)


def select_tour(dist, records, cost):
    """The DP's tie rule over the optimal set (tspgpu_select_tour)."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    arr = (TourRecord * max(1, len(records)))(*records)
    tour = np.zeros(n + 1, dtype=np.int32)
    rc = lib().tspgpu_select_tour(d.ctypes.data, dt, n, arr, len(records), cost_bits(cost, dt), _ip(tour))
    if rc:
        raise TspGpuError(rc, "tspgpu_select_tour")
    return tour


def tie_key(tour):
    """The device tie rule's key (w0, w1) of a tour 0, t1..tN, 0 (tspgpu_tie_key)."""
    t = np.ascontiguousarray(tour, dtype=np.int32)
    w0, w1 = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().tspgpu_tie_key(len(t) - 1, _ip(t), ctypes.byref(w0), ctypes.byref(w1))
    if rc:
        raise TspGpuError(rc, "tspgpu_tie_key")
    return w0.value, w1.value


def tie_tour(dist, w0: int, w1: int, cost):
    """Decode + certify a tie key (tspgpu_tie_tour): (rc, tour); rc 0 = tsp()'s
    tour, -EAGAIN = a tour of that cost the DP may not pick."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    tour = np.zeros(n + 1, dtype=np.int32)
    rc = lib().tspgpu_tie_tour(d.ctypes.data, dt, n, w0, w1, cost_bits(cost, dt), _ip(tour))
    return rc, tour


def tie_tour_gpu(ctx: "Context", dist, w0: int, w1: int, cost):
    """tie_tour with the certificate's prefix DPs on the context's GPU
    (tspgpu_tie_tour_gpu): (rc, tour)."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    tour = np.zeros(n + 1, dtype=np.int32)
    rc = lib().tspgpu_tie_tour_gpu(ctx.handle, d.ctypes.data, dt, n, w0, w1, cost_bits(cost, dt), _ip(tour))
    return rc, tour


def tie_tour_records(ctx, dist, w0: int, w1: int, cost, records):
    """tie_tour with the certificate's prefix minima from the search's records
    (tspgpu_tie_tour_records): `records` must be every tour the search
    recorded at the optimum (Search.records(opt) without overflow, all
    shards).  ctx: the GPU DP for a prefix the records cannot decide (None:
    not certified).  -> (rc, tour)."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    tour = np.zeros(n + 1, dtype=np.int32)
    arr = (TourRecord * max(1, len(records)))(*records)
    rc = lib().tspgpu_tie_tour_records(ctx.handle if ctx is not None else None, d.ctypes.data, dt, n, w0, w1,
                                       cost_bits(cost, dt), arr, len(records), _ip(tour))
    return rc, tour


class Search:
    """One instance (or shard `shard` of `nshards`) of the K2 search on a Context."""

    def __init__(self, ctx: "Context", dist, shard: int = 0, nshards: int = 1, depth: int = 0,
                 device_bound: bool = False):
        """device_bound: the initial incumbent from the create launch's device
        heuristic (TSPGPU_SEARCH_DEVICE_BOUND) instead of set_bound."""
        self.dist, self.dtype = _search_dist(dist)
        self.n = self.dist.shape[0]
        h = ctypes.c_void_p()
        rc = lib().tspgpu_search_create_ex(ctx.handle, self.dist.ctypes.data, self.dtype, self.n, shard, nshards,
                                           depth, 1 if device_bound else 0, ctypes.byref(h))
        if rc:
            raise TspGpuError(rc, "tspgpu_search_create_ex")
        self.handle = h
        dep, items, local = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        lib().tspgpu_search_info(h, ctypes.byref(dep), ctypes.byref(items), ctypes.byref(local))
        self.depth, self.items, self.local_items = dep.value, items.value, local.value

    def close(self):
        if self.handle:
            lib().tspgpu_search_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc:
            raise TspGpuError(rc, what)

    def set_bound(self, bound: float):
        self._check(lib().tspgpu_search_set_bound(self.handle, float(bound)), "tspgpu_search_set_bound")

    def start(self):
        """Seed this shard's live prefixes."""
        self._check(lib().tspgpu_search_start(self.handle), "tspgpu_search_start")

    def step(self) -> int:
        """One round; returns the items pending for the next round."""
        p = ctypes.c_uint64()
        self._check(lib().tspgpu_search_step(self.handle, ctypes.byref(p)), "tspgpu_search_step")
        return p.value

    def run_all(self):
        self._check(lib().tspgpu_search_run_all(self.handle), "tspgpu_search_run_all")

    def chain(self, exchange_every: int = 0, hook=None, native_hook=None) -> bool:
        """This shard's whole search chained on the device with one
        synchronisation (tspgpu_search_chain); False: not a chain (too large:
        the shard is at its starting state; or too small to have a frontier
        level) — continue with start/step.  Every `exchange_every` levels an
        exchange of the device incumbent word is enqueued on the search's
        stream, by hook(stream, word) (Python) or native_hook = (address of a
        C tspgpu_level_hook, its user pointer), e.g. libtspcomm's in-stream
        RCCL all-reduce MIN; the same count on every shard either way."""
        done = ctypes.c_int()
        user = None
        if native_hook is not None:
            cb, user = LEVEL_HOOK(native_hook[0]), native_hook[1]
        elif hook is not None:
            cb = LEVEL_HOOK(lambda _u, st, w: hook(st, w))
        else:
            cb = LEVEL_HOOK()
        every = exchange_every if (hook is not None or native_hook is not None) else 0
        self._check(lib().tspgpu_search_chain(self.handle, every, cb, user, ctypes.byref(done)),
                    "tspgpu_search_chain")
        return bool(done.value)

    def tie_slot(self, bits: int):
        """The device tie rule's least key at cost word `bits` on this shard:
        (found, w0, w1, overflow)."""
        t = TieSlot()
        self._check(lib().tspgpu_search_tie_slot(self.handle, bits, ctypes.byref(t)), "tspgpu_search_tie_slot")
        return bool(t.found), int(t.w0), int(t.w1), bool(t.overflow)

    def timing(self):
        ms, rounds = ctypes.c_double(), ctypes.c_int()
        self._check(lib().tspgpu_search_timing(self.handle, ctypes.byref(ms), ctypes.byref(rounds)),
                    "tspgpu_search_timing")
        return ms.value, rounds.value

    @property
    def incumbent_ptr(self) -> int:
        return lib().tspgpu_search_incumbent_device(self.handle)

    def counters(self):
        inc, nodes, recs = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(lib().tspgpu_search_counters(self.handle, ctypes.byref(inc), ctypes.byref(nodes),
                                                 ctypes.byref(recs)), "tspgpu_search_counters")
        return inc.value, nodes.value, recs.value

    def reset_records(self, capacity: int = 0):
        self._check(lib().tspgpu_search_reset_records(self.handle, capacity), "tspgpu_search_reset_records")

    def records(self, bits: int):
        """Recorded tours whose cost word equals `bits` (list of TourRecord)."""
        cnt = ctypes.c_int()
        rc = lib().tspgpu_search_records(self.handle, bits, None, 0, ctypes.byref(cnt))
        if rc and rc != -errno.ENOSPC:
            raise TspGpuError(rc, "tspgpu_search_records")
        arr = (TourRecord * max(1, cnt.value))()
        self._check(lib().tspgpu_search_records(self.handle, bits, arr, cnt.value, ctypes.byref(cnt)),
                    "tspgpu_search_records")
        return list(arr[:cnt.value])


def search_solve(ctx: "Context", dist, exhaustive: bool = False):
    """One instance on one GPU: (cost, tour (n+1,), stats dict).  exhaustive:
    enumerate every tour (no bound; tspgpu_search_enumerate)."""
    d, dt = _search_dist(dist)
    n = d.shape[0]
    cost = ctypes.c_double()
    tour = np.zeros(n + 1, dtype=np.int32)
    st = SearchStats()
    fn = lib().tspgpu_search_enumerate if exhaustive else lib().tspgpu_search_solve
    rc = fn(ctx.handle, d.ctypes.data, dt, n, ctypes.byref(cost), _ip(tour), ctypes.byref(st))
    if rc:
        raise TspGpuError(rc, "tspgpu_search_enumerate" if exhaustive else "tspgpu_search_solve")
    c = cost.value if dt == F64 else int(cost.value)
    return c, tour, st.as_dict()


def errno_name(code: int) -> str:
    return errno.errorcode.get(-code, str(code))
