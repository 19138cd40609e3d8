// Start-up costs of the drop-in, phase by phase (development aid): the HIP
// runtime, a context, and the FIRST use of each kernel family (its code
// object's load) next to a second use, through the C ABI.
//   hipcc -O2 -I include tools/init_probe2.cpp -L tsp-mpi-reduction_amd/lib -ltspgpu \
//       -Wl,-rpath,$PWD/tsp-mpi-reduction_amd/lib -o tsp-mpi-reduction_amd/bin/init_probe2
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

__global__ void probe_nop(int *p)
{
    if (p) *p = 1;
}

static std::vector<double> instance(int n, int seed)
{
    std::vector<tspgpu_city> c(n);
    unsigned s = 12345u + seed;
    for (int i = 0; i < n; ++i) {
        s = s * 1103515245u + 12345u;
        c[i].id = i;
        c[i].x = (s >> 8) % 1000;
        s = s * 1103515245u + 12345u;
        c[i].y = (s >> 8) % 1000 + 0.5;
    }
    std::vector<double> d((size_t)n * n);
    tspgpu_distance_matrix(c.data(), n, 1, d.data());
    return d;
}

int main()
{
    double t = now_ms();
    const double t00 = t;
    auto lap = [&](const char *what) {
        const double u = now_ms();
        std::printf("%-40s %8.2f ms\n", what, u - t);
        t = u;
    };
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    lap("hipGetDeviceCount (runtime init)");
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    lap("hipGetDeviceProperties");
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    lap("hipStreamCreateWithFlags");
    int *p = nullptr;
    (void)hipMalloc((void **)&p, 1 << 20);
    lap("hipMalloc 1 MB");
    hipLaunchKernelGGL(probe_nop, dim3(1), dim3(64), 0, st, p);
    (void)hipStreamSynchronize(st);
    lap("first launch, this binary's kernel");
    hipLaunchKernelGGL(probe_nop, dim3(1), dim3(64), 0, st, p);
    (void)hipStreamSynchronize(st);
    lap("second launch");
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    tspgpu_ctx *ctx = nullptr;
    if (tspgpu_ctx_create(&o, &ctx)) return 1;
    lap("tspgpu_ctx_create");
    std::vector<int32_t> tour(40);
    double cost = 0.0;
    for (int n : {5, 16, 16, 13, 13}) {
        const std::vector<double> d = instance(n, n);
        if (tspgpu_solve_blocks(ctx, d.data(), n, 1, &cost, tour.data())) return 1;
        char what[64];
        std::snprintf(what, sizeof what, "K1 one block, n = %d", n);
        lap(what);
    }
    for (int rep = 0; rep < 2; ++rep) {
        const std::vector<double> d = instance(16, 3);
        double c2 = 0.0;
        tspgpu_search_stats ss;
        std::memset(&ss, 0, sizeof ss);
        if (tspgpu_search_solve(ctx, d.data(), TSPGPU_F64, 16, &c2, tour.data(), &ss)) return 1;
        lap(rep ? "K2 search, 16 cities (again)" : "K2 search, 16 cities (first)");
    }
    {
        const int B = 4096, n = 16;
        std::vector<double> d((size_t)B * n * n);
        for (int b = 0; b < B; ++b) {
            const std::vector<double> x = instance(n, b);
            std::memcpy(d.data() + (size_t)b * n * n, x.data(), x.size() * sizeof(double));
        }
        std::vector<double> cs(B);
        std::vector<int32_t> ts((size_t)B * (n + 1));
        lap("(host: 4096 distance matrices)");
        for (int rep = 0; rep < 2; ++rep) {
            if (tspgpu_solve_blocks(ctx, d.data(), n, B, cs.data(), ts.data())) return 1;
            lap(rep ? "K1 4096 blocks n = 16 (again)" : "K1 4096 blocks n = 16 (first: sub-cube kernel)");
        }
    }
    tspgpu_ctx_destroy(ctx);
    lap("tspgpu_ctx_destroy");
    std::printf("%-40s %8.2f ms\n", "total", now_ms() - t00);
    return 0;
}
