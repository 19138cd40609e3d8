// How much of a latency-bound chained launch is one device-scope atomicAdd
// per block (development aid for the K2 expand levels, round 6): 200
// back-to-back launches of 512 blocks x 256 threads, each block (a) doing
// nothing but a load and a store, (b) the same plus thread 0's atomicAdd on a
// global counter whose result every thread then uses, (c) a block-wide
// barrier pair around (b) as expand_kernel has it.  Prints us per launch.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_plain(const unsigned *in, unsigned *out)
{
    const unsigned v = in[blockIdx.x * 256 + threadIdx.x];
    out[blockIdx.x * 256 + threadIdx.x] = v + 1;
}
__global__ void k_atomic(const unsigned *in, unsigned *out, unsigned *ctr)
{
    __shared__ unsigned base;
    const unsigned v = in[blockIdx.x * 256 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) base = atomicAdd(ctr, 1u);
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = v + base;
}
__global__ void k_load_chain(const unsigned *in, unsigned *out, const unsigned *cnt)
{
    // a device-scope load of a count first (as a chained level reads its input count)
    const unsigned c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned v = in[(blockIdx.x * 256 + threadIdx.x + c) & (512 * 256 - 1)];
    out[blockIdx.x * 256 + threadIdx.x] = v + 1;
}

__global__ void k_atomic_spread(const unsigned *in, unsigned *out, unsigned *ctr)
{
    // the same, each block on its own counter (no contention: latency only)
    __shared__ unsigned base;
    const unsigned v = in[blockIdx.x * 256 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) base = atomicAdd(ctr + 16 * blockIdx.x, 1u);
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = v + base;
}
__global__ void k_barriers(const unsigned *in, unsigned *out)
{
    __shared__ unsigned base;
    const unsigned v = in[blockIdx.x * 256 + threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) base = v;
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = v + base;
}

int main()
{
    unsigned *in, *out, *ctr;
    (void)hipMalloc(&in, 1024 * 256 * 4);
    (void)hipMalloc(&out, 1024 * 256 * 4);
    (void)hipMalloc(&ctr, 1024 * 64);
    (void)hipMemset(in, 0, 1024 * 256 * 4);
    (void)hipMemset(ctr, 0, 1024 * 64);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 20; ++w) launch();
        (void)hipStreamSynchronize(s);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a, s);
        for (int i = 0; i < 200; ++i) launch();
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        std::printf("%-40s %7.2f us per launch\n", name, ms * 1e3 / 200);
    };
    for (int g : {64, 256, 512, 1024}) {
        char nm[96];
        std::printf("grid %d blocks of 256\n", g);
        std::snprintf(nm, sizeof nm, "  load + store");
        run(nm, [&] { hipLaunchKernelGGL(k_plain, dim3(g), dim3(256), 0, s, in, out); });
        std::snprintf(nm, sizeof nm, "  + two block barriers");
        run(nm, [&] { hipLaunchKernelGGL(k_barriers, dim3(g), dim3(256), 0, s, in, out); });
        std::snprintf(nm, sizeof nm, "  count load first (device scope)");
        run(nm, [&] { hipLaunchKernelGGL(k_load_chain, dim3(g), dim3(256), 0, s, in, out, ctr); });
        std::snprintf(nm, sizeof nm, "  atomicAdd, one counter");
        run(nm, [&] { hipLaunchKernelGGL(k_atomic, dim3(g), dim3(256), 0, s, in, out, ctr); });
        std::snprintf(nm, sizeof nm, "  atomicAdd, a counter per block");
        run(nm, [&] { hipLaunchKernelGGL(k_atomic_spread, dim3(g), dim3(256), 0, s, in, out, ctr); });
    }
    return 0;
}
