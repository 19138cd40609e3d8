// Small transfers through mapped pinned slots and our own copy kernel (xfer.h).
#include "xfer.h"

#include <cstdint>
#include <cstring>
#include <mutex>

namespace tspgpu {
namespace {

// word-granular copy / fill; W = the widest word both ends are aligned to
template <typename W>
__global__ __launch_bounds__(256) void xcopy_kernel(const W *__restrict__ src, W *__restrict__ dst, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
template <typename W>
__global__ __launch_bounds__(256) void xset_kernel(W *__restrict__ dst, W v, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = v;
}

int grid_for(size_t n) { return (int)(n / 256 + 1 < 1024 ? n / 256 + 1 : 1024); }

hipError_t launch_copy(const void *src, void *dst, size_t bytes, hipStream_t st)
{
    const uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)bytes;
    if (!(a & 15)) {
        hipLaunchKernelGGL(xcopy_kernel<uint4>, dim3(grid_for(bytes / 16)), dim3(256), 0, st,
                           static_cast<const uint4 *>(src), static_cast<uint4 *>(dst), bytes / 16);
    } else if (!(a & 7)) {
        hipLaunchKernelGGL(xcopy_kernel<uint64_t>, dim3(grid_for(bytes / 8)), dim3(256), 0, st,
                           static_cast<const uint64_t *>(src), static_cast<uint64_t *>(dst), bytes / 8);
    } else if (!(a & 3)) {
        hipLaunchKernelGGL(xcopy_kernel<uint32_t>, dim3(grid_for(bytes / 4)), dim3(256), 0, st,
                           static_cast<const uint32_t *>(src), static_cast<uint32_t *>(dst), bytes / 4);
    } else {
        hipLaunchKernelGGL(xcopy_kernel<uint8_t>, dim3(grid_for(bytes)), dim3(256), 0, st,
                           static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), bytes);
    }
    return hipGetLastError();
}

// the slot pool: process-wide, any device (portable mapped pinned memory)
constexpr int kSlots = 8;
struct Slot {
    char *h = nullptr;
    hipEvent_t ev = nullptr;  // behind the last kernel that read or wrote the slot
    int dev = -1;             // device of ev
    bool pending = false;
};
struct Pool {
    std::mutex mu;
    Slot s[kSlots];
    int next = 0;
    bool broken = false;  // pinned allocation failed once: always the runtime path
};
Pool &pool()
{
    static Pool p;
    return p;
}

// a free slot (waiting for its last user if all are busy), or null
Slot *take(Pool &p, int dev)
{
    if (p.broken) return nullptr;
    Slot &s = p.s[p.next];
    p.next = (p.next + 1) % kSlots;
    if (!s.h) {
        if (hipHostMalloc((void **)&s.h, kXferSlotBytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
            s.h = nullptr;
            p.broken = true;
            return nullptr;
        }
    }
    if (s.pending) {
        if (hipEventSynchronize(s.ev) != hipSuccess) return nullptr;
        s.pending = false;
    }
    if (s.dev != dev) {
        if (s.ev) (void)hipEventDestroy(s.ev);
        s.ev = nullptr;
        if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
            s.ev = nullptr;
            s.dev = -1;
            return nullptr;
        }
        s.dev = dev;
    }
    return &s;
}

}  // namespace

hipError_t xcopy_async(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    if (kind == hipMemcpyDeviceToDevice) return launch_copy(src, dst, bytes, st);
    if (bytes > kXferSlotBytes || (kind != hipMemcpyHostToDevice && kind != hipMemcpyDeviceToHost))
        return hipMemcpyAsync(dst, src, bytes, kind, st);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    Pool &p = pool();
    std::lock_guard<std::mutex> g(p.mu);
    Slot *s = take(p, dev);
    if (!s) return hipMemcpyAsync(dst, src, bytes, kind, st);
    if (kind == hipMemcpyHostToDevice) {
        std::memcpy(s->h, src, bytes);
        e = launch_copy(s->h, dst, bytes, st);
        if (e == hipSuccess) e = hipEventRecord(s->ev, st);
        s->pending = e == hipSuccess;
        return e;
    }
    e = launch_copy(src, s->h, bytes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) std::memcpy(dst, s->h, bytes);
    return e;
}

hipError_t xset_async(void *dst, int value, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    const uint32_t b = (uint32_t)value & 0xffu;
    if (!(((uintptr_t)dst | bytes) & 3)) {
        hipLaunchKernelGGL(xset_kernel<uint32_t>, dim3(grid_for(bytes / 4)), dim3(256), 0, st,
                           static_cast<uint32_t *>(dst), b * 0x01010101u, bytes / 4);
    } else {
        hipLaunchKernelGGL(xset_kernel<uint8_t>, dim3(grid_for(bytes)), dim3(256), 0, st,
                           static_cast<uint8_t *>(dst), (uint8_t)b, bytes);
    }
    return hipGetLastError();
}

}  // namespace tspgpu
