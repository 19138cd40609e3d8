// Launch-cost probe (gfx950): near-empty kernels of different shapes and LDS
// sizes, event-timed, to separate fixed per-launch costs from kernel work.
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

template <int LDSB>
__global__ __launch_bounds__(256) void k_static(const unsigned short *in, int *out)
{
    __shared__ unsigned short s[LDSB / 2 > 0 ? LDSB / 2 : 1];
    for (int i = threadIdx.x; i < 1024; i += 256) s[i % (LDSB / 2 > 0 ? LDSB / 2 : 1)] = in[i];
    __syncthreads();
    if (s[threadIdx.x % (LDSB / 2 > 0 ? LDSB / 2 : 1)] == 12345) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_dyn(const unsigned short *in, int *out)
{
    extern __shared__ unsigned short s[];
    for (int i = threadIdx.x; i < 1024; i += 256) s[i] = in[i];
    __syncthreads();
    if (s[threadIdx.x] == 12345) out[0] = 1;
}

template <typename F>
void timeit(const char *name, F launch)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 10; ++r) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("%-40s %.4f ms/launch\n", name, ms / 10);
}

int main()
{
    unsigned short *in;
    int *out;
    CHECK(hipMalloc(&in, 1 << 16));
    CHECK(hipMemset(in, 0, 1 << 16));
    CHECK(hipMalloc(&out, 64));
    timeit("static 44KB, 768 x 256", [&] { hipLaunchKernelGGL(k_static<44032>, dim3(768), dim3(256), 0, 0, in, out); });
    timeit("static 4KB, 768 x 256", [&] { hipLaunchKernelGGL(k_static<4096>, dim3(768), dim3(256), 0, 0, in, out); });
    timeit("dynamic 44KB, 768 x 256", [&] { hipLaunchKernelGGL(k_dyn, dim3(768), dim3(256), 44032, 0, in, out); });
    timeit("dynamic 4KB, 768 x 256", [&] { hipLaunchKernelGGL(k_dyn, dim3(768), dim3(256), 4096, 0, in, out); });
    timeit("static 44KB, 16384 x 256", [&] { hipLaunchKernelGGL(k_static<44032>, dim3(16384), dim3(256), 0, 0, in, out); });
    return 0;
}
