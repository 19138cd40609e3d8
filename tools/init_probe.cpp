// Where the drop-in's process time goes (development aid): phases of a
// one-block 16-city solve through the C ABI, each with its own clock.
//   hipcc -O2 -I include tools/init_probe.cpp -L tsp-mpi-reduction_amd/lib -ltspgpu \
//       -Wl,-rpath,$PWD/tsp-mpi-reduction_amd/lib -o tsp-mpi-reduction_amd/bin/init_probe
//   init_probe [plain]   ("plain": HIP runtime only, no libtspgpu call)
#include <hip/hip_runtime.h>
#include <time.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#ifndef PLAIN
#include "tspgpu.h"
#endif

static double now_ms()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int main(int argc, char **argv)
{
    const bool plain = argc > 1 && std::strcmp(argv[1], "plain") == 0;
    double t = now_ms();
    auto lap = [&](const char *what) {
        const double u = now_ms();
        std::printf("%-28s %8.2f ms\n", what, u - t);
        t = u;
    };
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    lap("hipGetDeviceCount");
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    lap("hipSetDevice + hipFree(0)");
    if (plain) return 0;
#ifndef PLAIN  // -DPLAIN: a binary that does not link libtspgpu at all
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    tspgpu_ctx *ctx = nullptr;
    if (tspgpu_ctx_create(&o, &ctx)) return 1;
    lap("tspgpu_ctx_create");
    const int n = 16;
    std::vector<double> d(n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) d[i * n + j] = std::fabs(std::sin(i * 7.0 + j * 3.0)) * 100.0 + (i == j ? 0 : 1);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) d[i * n + j] = d[j * n + i];
    for (int i = 0; i < n; ++i) d[i * n + i] = 0.0;
    double cost = 0.0;
    std::vector<int32_t> tour(n + 1);
    for (int rep = 0; rep < 3; ++rep) {
        if (tspgpu_solve_blocks(ctx, d.data(), n, 1, &cost, tour.data())) return 1;
        lap(rep == 0 ? "first solve (16 cities)" : "next solve");
    }
    tspgpu_ctx_destroy(ctx);
    lap("tspgpu_ctx_destroy");
    std::printf("cost %.6f\n", cost);
#endif
    return 0;
}
