// Chain-cost probe (gfx950, development aid): what a chain of small dependent
// launches costs on the device, against one launch whose blocks meet at
// grid-wide barriers between "levels" — the question behind K2's chained
// frontier levels (~11 us each at 16 cities whatever their work).
//   chain:   K back-to-back launches of a near-empty kernel (shape of
//            expand_kernel: 512 x 256, ~18 KB LDS), timed by two events
//            around all K (so one event pair, not one per launch)
//   barrier: one launch of G blocks (<= one per CU: all resident) running L
//            levels separated by a grid barrier (a device-scope counter, a
//            generation word; every spin is bounded: a block that waits too
//            long raises an error flag and the launch ends)
// hipcc --offload-arch=gfx950 -O3 tools/ubench_chain.hip -o bin/ubench_chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                                  \
        }                                                                             \
    } while (0)

__global__ __launch_bounds__(256) void k_level(const double *in, double *out, int early)
{
    __shared__ double s[2304];
    for (int i = threadIdx.x; i < 256; i += 256) s[i] = in[i];
    __syncthreads();
    if (early && blockIdx.x >= 32) return;
    if (s[threadIdx.x] == 12345.0) out[blockIdx.x] = 1.0;
}

// grid barrier: arrive = atomicAdd on count; the last arriver resets count
// and bumps gen; the others wait for gen to change (bounded)
__device__ bool grid_sync(unsigned int *count, unsigned int *gen, unsigned int *err, unsigned int nblocks)
{
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const unsigned int g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned int a = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (a == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            long spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > 20000000L) {  // ~ seconds: never expected; end the launch
                    __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
    }
    __shared__ int okb;
    if (threadIdx.x == 0) okb = ok;
    __syncthreads();
    return okb != 0;
}

__global__ __launch_bounds__(256) void k_levels(const double *in, double *out, unsigned int *sync, int levels)
{
    __shared__ double s[2304];
    for (int l = 0; l < levels; ++l) {
        for (int i = threadIdx.x; i < 256; i += 256) s[i] = in[i] + l;
        __syncthreads();
        if (s[threadIdx.x] == 12345.0) out[blockIdx.x] = 1.0;
        if (!grid_sync(sync, sync + 1, sync + 2, gridDim.x)) return;
    }
}

int main()
{
    double *in, *out;
    unsigned int *sync;
    CHECK(hipMalloc(&in, 1 << 16));
    CHECK(hipMemset(in, 0, 1 << 16));
    CHECK(hipMalloc(&out, 1 << 16));
    CHECK(hipMalloc(&sync, 64));
    CHECK(hipMemset(sync, 0, 64));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct Shape {
        int grid, early;
        const char *name;
    } shapes[] = {{1, 0, "1 block"}, {512, 0, "512 blocks"}, {512, 1, "512 blocks, 480 leave early"},
                  {2048, 1, "2048 blocks, 2016 leave early"}};
    for (const Shape &sh : shapes)
        for (int K : {1, 5, 10}) {
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipStreamSynchronize(st));
                CHECK(hipEventRecord(a, st));
                for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_level, dim3(sh.grid), dim3(256), 0, st, in, out, sh.early);
                CHECK(hipEventRecord(b, st));
                CHECK(hipEventSynchronize(b));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, a, b));
                if (rep == 1) printf("chain   %-32s K=%2d  %.2f us total  %.2f us/launch\n", sh.name, K, ms * 1e3, ms * 1e3 / K);
            }
        }
    for (int G : {64, 128, 256}) {
        if (G > cus) continue;
        for (int L : {1, 5, 10}) {
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipMemsetAsync(sync, 0, 64, st));
                CHECK(hipStreamSynchronize(st));
                CHECK(hipEventRecord(a, st));
                hipLaunchKernelGGL(k_levels, dim3(G), dim3(256), 0, st, in, out, sync, L);
                CHECK(hipEventRecord(b, st));
                CHECK(hipEventSynchronize(b));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, a, b));
                unsigned int h[3];
                CHECK(hipMemcpy(h, sync, sizeof h, hipMemcpyDeviceToHost));
                if (rep == 1)
                    printf("barrier %3d blocks L=%2d  %.2f us total  %.2f us/level  err=%u\n", G, L, ms * 1e3, ms * 1e3 / L, h[2]);
                if (h[2]) return 3;
            }
        }
    }
    return 0;
}
