// Which first-use HIP costs the drop-in pays before its first answer
// (development aid, round 5): stream creation vs the null stream, the first
// pageable vs pinned upload, a pinned allocation.  One process per mode:
//   init_probe3 stream | null | pinned
#include <hip/hip_runtime.h>
#include <time.h>

#include <cstdio>
#include <cstring>
#include <vector>

static double now_ms()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

__global__ void probe_add(int *p)
{
    p[threadIdx.x] += 1;
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "stream";
    double t = now_ms();
    auto lap = [&](const char *what) {
        const double u = now_ms();
        std::printf("%-8s %-36s %8.2f ms\n", mode, what, u - t);
        t = u;
    };
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    lap("hipGetDeviceCount (runtime init)");
    hipStream_t st = nullptr;
    if (std::strcmp(mode, "null") != 0) {
        (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        lap("hipStreamCreateWithFlags");
    }
    int *d = nullptr;
    (void)hipMalloc((void **)&d, 1 << 20);
    lap("hipMalloc 1 MB");
    std::vector<int> h(1 << 16, 1);
    int *hp = h.data();
    if (std::strcmp(mode, "pinned") == 0) {
        (void)hipHostMalloc((void **)&hp, (1 << 16) * sizeof(int), hipHostMallocDefault);
        lap("hipHostMalloc 256 KB");
        std::memcpy(hp, h.data(), (1 << 16) * sizeof(int));
    }
    (void)hipMemcpyAsync(d, hp, (1 << 16) * sizeof(int), hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
    lap("first upload 256 KB");
    (void)hipMemcpyAsync(d, hp, (1 << 16) * sizeof(int), hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
    lap("second upload 256 KB");
    hipLaunchKernelGGL(probe_add, dim3(1), dim3(64), 0, st, d);
    (void)hipStreamSynchronize(st);
    lap("first launch");
    (void)hipMemcpyAsync(hp, d, 256, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    lap("first readback 256 B");
    (void)hipMemcpyAsync(hp, d, 256, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    lap("second readback 256 B");
    return hp[0] == 2 ? 0 : 1;
}
