// Small transfers through mapped pinned slots and our own copy kernel (xfer.h).
#include "xfer.h"
#include "xfer_pool.h"

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

// hipLaunchKernel returns THIS launch's status (hipGetLastError after a
// triple-chevron launch would also return, and clear, an error some earlier
// call left on the thread)
template <typename W>
hipError_t launch_copy_w(const void *src, void *dst, size_t n, hipStream_t st)
{
    const W *s = static_cast<const W *>(src);
    W *d = static_cast<W *>(dst);
    void *args[] = {&s, &d, &n};
    return hipLaunchKernel(reinterpret_cast<const void *>(&xcopy_kernel<W>), dim3(grid_for(n)), dim3(256), args, 0, st);
}
hipError_t launch_copy(const void *src, void *dst, size_t bytes, hipStream_t st)
{
    const uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)bytes;
    if (!(a & 15)) return launch_copy_w<uint4>(src, dst, bytes / 16, st);
    if (!(a & 7)) return launch_copy_w<uint64_t>(src, dst, bytes / 8, st);
    if (!(a & 3)) return launch_copy_w<uint32_t>(src, dst, bytes / 4, st);
    return launch_copy_w<uint8_t>(src, dst, bytes, st);
}
template <typename W>
hipError_t launch_set_w(void *dst, W v, size_t n, hipStream_t st)
{
    W *d = static_cast<W *>(dst);
    void *args[] = {&d, &v, &n};
    return hipLaunchKernel(reinterpret_cast<const void *>(&xset_kernel<W>), dim3(grid_for(n)), dim3(256), args, 0, st);
}

// the pinned slots (xfer_pool.h): one pool per device, events of that device
struct HipSlots {
    using Event = hipEvent_t;
    using Stream = hipStream_t;
    template <typename S>
    bool alloc(S &s)
    {
        if (hipHostMalloc((void **)&s.h, kXferSlotBytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
            s.h = nullptr;
            return false;
        }
        if (hipEventCreateWithFlags(&s.ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipHostFree(s.h);
            s.h = nullptr;
            s.ev = nullptr;
            return false;
        }
        return true;
    }
    bool done(hipEvent_t e) { return hipEventQuery(e) == hipSuccess; }
};
constexpr int kMaxPoolDevs = 64;
using Pool = XferPool<HipSlots>;
Pool *pool(int dev)
{
    static Pool pools[kMaxPoolDevs];
    return dev >= 0 && dev < kMaxPoolDevs ? &pools[dev] : nullptr;
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
    Pool *p = pool(dev);
    bool wait = false;
    Pool::Slot *s = p ? p->claim(st, &wait) : nullptr;
    if (!s) return hipMemcpyAsync(dst, src, bytes, kind, st);
    // (outside the pool's lock: the slot is this thread's until release)
    if (wait) e = hipEventSynchronize(s->ev);  // the last copy through it, on this same stream
    if (e != hipSuccess) {
        p->release(s, st, true);
        return e;
    }
    if (kind == hipMemcpyHostToDevice) {
        std::memcpy(s->h, src, bytes);
        e = launch_copy(s->h, dst, bytes, st);
        if (e == hipSuccess) e = hipEventRecord(s->ev, st);
        p->release(s, st, e == hipSuccess);
        return e;
    }
    e = launch_copy(src, s->h, bytes, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) std::memcpy(dst, s->h, bytes);
    p->release(s, st, false);
    return e;
}

hipError_t xset_async(void *dst, int value, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    const uint32_t b = (uint32_t)value & 0xffu;
    if (!(((uintptr_t)dst | bytes) & 3)) return launch_set_w<uint32_t>(dst, b * 0x01010101u, bytes / 4, st);
    return launch_set_w<uint8_t>(dst, (uint8_t)b, bytes, st);
}

}  // namespace tspgpu
