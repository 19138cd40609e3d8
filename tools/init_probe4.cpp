// What the first 16-city solve pays (development aid, round 5): the first
// copy of the process, pageable and pinned copies of the K1 table size, a
// copy done by our own kernel from mapped pinned memory, and then the
// library's first n = 16 one-block solve once the copy path is warm.
//   init_probe4 raw | lib
#include <hip/hip_runtime.h>
#include <time.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "tspgpu.h"

static double now_ms()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

__global__ void probe_copy(const uint4 *src, uint4 *dst, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "raw";
    double t = now_ms();
    auto lap = [&](const char *what) {
        const double u = now_ms();
        std::printf("%-5s %-48s %8.2f ms\n", mode, what, u - t);
        t = u;
    };
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    lap("hipGetDeviceCount (runtime init)");
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    lap("hipStreamCreateWithFlags");
    const size_t B = 128 << 10;
    void *d = nullptr;
    (void)hipMalloc(&d, B);
    std::vector<char> h(B, 1);
    if (std::strcmp(mode, "raw") == 0) {
        void *hp = nullptr, *dp = nullptr;
        (void)hipHostMalloc(&hp, B, hipHostMallocMapped);
        (void)hipHostGetDevicePointer(&dp, hp, 0);
        std::memcpy(hp, h.data(), B);
        lap("hipHostMalloc mapped 128 KB");
        hipLaunchKernelGGL(probe_copy, dim3(32), dim3(256), 0, st, (const uint4 *)dp, (uint4 *)d, B / 16);
        (void)hipStreamSynchronize(st);
        lap("kernel copy 128 KB from mapped pinned (first launch)");
        hipLaunchKernelGGL(probe_copy, dim3(32), dim3(256), 0, st, (const uint4 *)dp, (uint4 *)d, B / 16);
        (void)hipStreamSynchronize(st);
        lap("kernel copy 128 KB again");
        (void)hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
        lap("hipMemcpy 4 KB pageable (first copy)");
        (void)hipMemcpy(d, h.data(), B, hipMemcpyHostToDevice);
        lap("hipMemcpy 128 KB pageable");
        (void)hipMemcpy(d, h.data(), B, hipMemcpyHostToDevice);
        lap("hipMemcpy 128 KB pageable again");
        (void)hipMemcpy(d, hp, B, hipMemcpyHostToDevice);
        lap("hipMemcpy 128 KB pinned");
        (void)hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
        lap("hipMemcpy 4 KB D2H");
        (void)hipMemsetAsync(d, 0xff, 4096, st);
        (void)hipStreamSynchronize(st);
        lap("hipMemsetAsync 4 KB (first fill)");
        return 0;
    }
    (void)hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
    (void)hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost);
    (void)hipMemsetAsync(d, 0xff, 4096, st);
    (void)hipStreamSynchronize(st);
    lap("first copies + fill (warm the copy path)");
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    tspgpu_ctx *ctx = nullptr;
    if (tspgpu_ctx_create(&o, &ctx)) return 1;
    lap("tspgpu_ctx_create");
    const int n = 16;
    std::vector<tspgpu_city> c(n);
    unsigned s = 12345u;
    for (int i = 0; i < n; ++i) {
        s = s * 1103515245u + 12345u;
        c[i] = {i, (double)((s >> 8) % 1000), (double)((s >> 12) % 1000)};
    }
    std::vector<double> dist((size_t)n * n);
    tspgpu_distance_matrix(c.data(), n, 1, dist.data());
    std::vector<int32_t> tour(n + 1);
    double cost = 0.0;
    for (int rep = 0; rep < 3; ++rep) {
        if (tspgpu_solve_blocks(ctx, dist.data(), n, 1, &cost, tour.data())) return 1;
        lap(rep ? "K1 one block n = 16 (again)" : "K1 one block n = 16 (first)");
    }
    tspgpu_ctx_destroy(ctx);
    lap("tspgpu_ctx_destroy");
    return 0;
}
