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
LIB_PATH = os.path.join(PKG_DIR, "lib", "libtspgpu.so")
HOST_LIB_PATH = os.path.join(PKG_DIR, "lib", "libtsphost.so")
TSP_BIN = os.path.join(PKG_DIR, "bin", "tsp")

EXPORTED_SYMBOLS = (
    "tspgpu_version", "tspgpu_strerror", "tspgpu_tour_length", "tspgpu_distance_matrix", "tspgpu_validate",
    "tspgpu_ctx_create", "tspgpu_ctx_destroy", "tspgpu_solve_blocks", "tspgpu_solve_cities",
    "tspgpu_solve_blocks_device", "tspgpu_solve", "tspgpu_last_grid", "tspgpu_relaxations_per_block",
    "tspgpu_table_bytes_per_block", "tspgpu_device_alloc", "tspgpu_device_free", "tspgpu_memcpy_htod",
    "tspgpu_memcpy_dtoh", "tspgpu_stream", "tspgpu_synchronize", "tspgpu_timer_start", "tspgpu_timer_stop",
    "tspgpu_device_info",
)


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
        L.tspgpu_solve.argtypes = [dp, ctypes.c_int, ctypes.c_int, dp, ip, ctypes.POINTER(Opts)]
        L.tspgpu_last_grid.argtypes = [vp]
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
        L.tspgpu_timer_start.argtypes = [vp]
        L.tspgpu_timer_stop.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
        L.tspgpu_device_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


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

    def synchronize(self):
        self._check(lib().tspgpu_synchronize(self.handle), "tspgpu_synchronize")

    def timer_start(self):
        self._check(lib().tspgpu_timer_start(self.handle), "tspgpu_timer_start")

    def timer_stop(self) -> float:
        ms = ctypes.c_float()
        self._check(lib().tspgpu_timer_stop(self.handle, ctypes.byref(ms)), "tspgpu_timer_stop")
        return ms.value

    def device_info(self):
        cu = ctypes.c_int()
        name = ctypes.create_string_buffer(256)
        self._check(lib().tspgpu_device_info(self.handle, ctypes.byref(cu), name, 256), "tspgpu_device_info")
        return cu.value, name.value.decode()


def errno_name(code: int) -> str:
    return errno.errorcode.get(-code, str(code))
